/*
 * ORACLE (test infrastructure only) — plain-C sparse LDL^T, the algorithm of
 * LDLFactorizations.jl 0.10.1 (the `LDLSolver` the reference's tests plug in,
 * /root/reference/test/runtests.jl:128,185; is_factorized at src/utils.jl:57-59), which is a
 * translation of T. A. Davis' "LDL" up-looking factorisation (ACM TOMS 31(4), 2005):
 * symbolic: elimination tree + column counts by row-subtree traversal; numeric: for every row k,
 * a sparse triangular solve L(0:k-1,0:k-1) y = A(0:k-1,k) over the reach of row k in the etree,
 * then L(k,:) = y ./ D, D(k) = A(k,k) - y' L(k,:)'.  No pivoting (static order P).
 * Unavailable dependency restated; LDLFactorizations itself is not in the container.
 *
 * Only tests/ and bench.py's cpu_baseline leg may load this (built to oracle/_build/).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  int64_t n;
  int64_t *Lp;   /* n+1 */
  int32_t *Li;   /* nnz(L) strictly lower */
  double *Lx;
  double *D;     /* n */
  int32_t *P, *Pinv, *Parent;
} ldl_ref_t;

/* Ap/Ai/Ax: full symmetric matrix in CSC (both triangles); P: permutation (P[k] = original index
 * of pivot k) or NULL for natural order. Returns NULL on allocation failure. */
ldl_ref_t* ldl_ref_symbolic(int64_t n, const int64_t* Ap, const int32_t* Ai, const int32_t* P) {
  ldl_ref_t* F = (ldl_ref_t*)calloc(1, sizeof(ldl_ref_t));
  if (!F) return NULL;
  F->n = n;
  F->Lp = (int64_t*)malloc(sizeof(int64_t) * (n + 1));
  F->P = (int32_t*)malloc(sizeof(int32_t) * (n > 0 ? n : 1));
  F->Pinv = (int32_t*)malloc(sizeof(int32_t) * (n > 0 ? n : 1));
  F->Parent = (int32_t*)malloc(sizeof(int32_t) * (n > 0 ? n : 1));
  int32_t* Flag = (int32_t*)malloc(sizeof(int32_t) * (n > 0 ? n : 1));
  int64_t* Lnz = (int64_t*)malloc(sizeof(int64_t) * (n > 0 ? n : 1));
  for (int64_t k = 0; k < n; ++k) F->P[k] = P ? P[k] : (int32_t)k;
  for (int64_t k = 0; k < n; ++k) F->Pinv[F->P[k]] = (int32_t)k;
  for (int64_t k = 0; k < n; ++k) {
    F->Parent[k] = -1;
    Flag[k] = (int32_t)k;
    Lnz[k] = 0;
    int64_t kk = F->P[k];
    for (int64_t p = Ap[kk]; p < Ap[kk + 1]; ++p) {
      int32_t i = F->Pinv[Ai[p]];
      if (i < k) {
        for (; Flag[i] != k; i = F->Parent[i]) {
          if (F->Parent[i] == -1) F->Parent[i] = (int32_t)k;
          Lnz[i]++;
          Flag[i] = (int32_t)k;
        }
      }
    }
  }
  F->Lp[0] = 0;
  for (int64_t k = 0; k < n; ++k) F->Lp[k + 1] = F->Lp[k] + Lnz[k];
  F->Li = (int32_t*)malloc(sizeof(int32_t) * (F->Lp[n] > 0 ? F->Lp[n] : 1));
  F->Lx = (double*)malloc(sizeof(double) * (F->Lp[n] > 0 ? F->Lp[n] : 1));
  F->D = (double*)malloc(sizeof(double) * (n > 0 ? n : 1));
  free(Flag);
  free(Lnz);
  return F;
}

int64_t ldl_ref_nnz(const ldl_ref_t* F) { return F->Lp[F->n]; }

/* Returns n on success, k if D(k) == 0 (factorisation stops there). */
int64_t ldl_ref_numeric(ldl_ref_t* F, const int64_t* Ap, const int32_t* Ai, const double* Ax) {
  const int64_t n = F->n;
  double* Y = (double*)calloc(n > 0 ? n : 1, sizeof(double));
  int32_t* Pattern = (int32_t*)malloc(sizeof(int32_t) * (n > 0 ? n : 1));
  int32_t* Flag = (int32_t*)malloc(sizeof(int32_t) * (n > 0 ? n : 1));
  int64_t* Lnz = (int64_t*)malloc(sizeof(int64_t) * (n > 0 ? n : 1));
  int64_t ret = n;
  for (int64_t k = 0; k < n; ++k) {
    Y[k] = 0.0;
    int64_t top = n;
    Flag[k] = (int32_t)k;
    Lnz[k] = 0;
    int64_t kk = F->P[k];
    for (int64_t p = Ap[kk]; p < Ap[kk + 1]; ++p) {
      int32_t i = F->Pinv[Ai[p]];
      if (i <= k) {
        Y[i] += Ax[p];
        int64_t len = 0;
        for (; Flag[i] != k; i = F->Parent[i]) {
          Pattern[len++] = i;
          Flag[i] = (int32_t)k;
        }
        while (len > 0) Pattern[--top] = Pattern[--len];
      }
    }
    F->D[k] = Y[k];
    Y[k] = 0.0;
    for (; top < n; ++top) {
      int32_t i = Pattern[top];
      double yi = Y[i];
      Y[i] = 0.0;
      int64_t p2 = F->Lp[i] + Lnz[i];
      for (int64_t p = F->Lp[i]; p < p2; ++p) Y[F->Li[p]] -= F->Lx[p] * yi;
      double l_ki = yi / F->D[i];
      F->D[k] -= l_ki * yi;
      F->Li[p2] = (int32_t)k;
      F->Lx[p2] = l_ki;
      Lnz[i]++;
    }
    if (F->D[k] == 0.0) {
      ret = k;
      break;
    }
  }
  free(Y);
  free(Pattern);
  free(Flag);
  free(Lnz);
  return ret;
}

/* x := A^{-1} b in the original ordering (in place), using the stored factors. */
void ldl_ref_solve(const ldl_ref_t* F, double* x) {
  const int64_t n = F->n;
  double* y = (double*)malloc(sizeof(double) * (n > 0 ? n : 1));
  for (int64_t k = 0; k < n; ++k) y[k] = x[F->P[k]];
  for (int64_t j = 0; j < n; ++j)
    for (int64_t p = F->Lp[j]; p < F->Lp[j + 1]; ++p) y[F->Li[p]] -= F->Lx[p] * y[j];
  for (int64_t j = 0; j < n; ++j) y[j] /= F->D[j];
  for (int64_t j = n - 1; j >= 0; --j)
    for (int64_t p = F->Lp[j]; p < F->Lp[j + 1]; ++p) y[j] -= F->Lx[p] * y[F->Li[p]];
  for (int64_t k = 0; k < n; ++k) x[F->P[k]] = y[k];
  free(y);
}

void ldl_ref_get_d(const ldl_ref_t* F, double* d) { memcpy(d, F->D, sizeof(double) * F->n); }

void ldl_ref_free(ldl_ref_t* F) {
  if (!F) return;
  free(F->Lp);
  free(F->Li);
  free(F->Lx);
  free(F->D);
  free(F->P);
  free(F->Pinv);
  free(F->Parent);
  free(F);
}
