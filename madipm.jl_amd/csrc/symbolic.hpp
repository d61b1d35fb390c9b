// Symbolic analysis for the multifrontal supernodal LDL^T (host side, runs once per pattern).
//
// Replaces the symbolic phase the reference's linear-solver constructor performs
// (`linear_solver(aug_com; opt)`, src/KKT/normalkkt.jl:113-115; MadNLP's SparseKKTSystem ctor for
// K2) — SURVEY §8 a12: fill-reducing ordering, elimination tree, column counts, fundamental +
// relaxed supernodes, frontal row structures, the assembly map from the caller's CSC values to
// frontal positions, child→parent relative indices and the level schedule used on the GPU.
#pragma once

#include <cstdint>
#include <atomic>
#include <vector>

#include "hvec.hpp"

namespace madipm {

// cap (optional): AMD stops early — returns false, perm empty — once a lower bound of its order's
// flops (sum (c - 1)(c + 2) over the column counts of the pivots eliminated so far) exceeds *cap, i.e.
// once it can no longer beat an order of *cap flops
bool amd_order(int n, const std::vector<int64_t>& Ap, const std::vector<int32_t>& Ai,
               std::vector<int32_t>& perm, double dense_alpha = 10.0, const std::atomic<double>* cap = nullptr);

struct NDOptions {
  int leaf_size = 256;       // subgraphs up to this size are ordered by AMD
  int tries = 3;             // multilevel bisections per subgraph (best separator kept)
  double sep_ratio = 0.1;    // a separator larger than this fraction => AMD for the subgraph
  double dense_alpha = 10.0; // for the AMD leaves
  int threads = 1;           // host threads for independent subgraphs / tries (the order does not depend on it)
  uint64_t seed = 12345;     // root of every subproblem's random stream
};

// Nested dissection (csrc/nd.cpp); same input convention as amd_order.
void nd_order(int n, const std::vector<int64_t>& Ap, const std::vector<int32_t>& Ai, std::vector<int32_t>& perm,
              const NDOptions& opt);

struct SymbolicOptions {
  int ordering = 1;          // 0: natural, 1: AMD, 2: user permutation, 3: nested dissection,
                             // 4: auto (AMD and ND, the one with fewer factorisation flops)
  double dense_alpha = 10.0; // AMD dense threshold = max(16, alpha*sqrt(n))
  int relax = 1;             // relaxed supernode amalgamation (zero-fraction rule) on/off
  int nrelax[3] = {4, 16, 48};
  double zrelax[3] = {0.8, 0.1, 0.05};
  // cost-based amalgamation of HBM-sized fronts (child rows > big_merge_rows): a child merges into
  // its parent when the update block it would write and its parent read back (16 B per entry) costs
  // more than the merge's extra trailing-update flops / big_merge (flops per byte, the f64 MFMA / HBM
  // ratio) plus the explicit zeros' traffic.  0 disables (env MADIPM_BIG_MERGE overrides).  Measured
  // (r5, profiles/r5_a_*): neos 31.5 -> 35.9 iters/s with 6; ex10 / supportcase10 have no front above
  // big_merge_rows and are unchanged.
  double big_merge = 6.0;
  int big_merge_rows = 256;
  int small_front_max = 128; // fronts with r <= this are factorised in LDS by one workgroup (max 192)
  int gather_max = 128;      // children with update blocks of more rows are added block-wise (bt), not gathered
  int fact_tree = 1;         // dependency-driven factorisation of the LDS-sized subtrees (k_fact_tree)
  // elimination-tree subtree sharding (SURVEY §8 e): the front tree is cut into independent
  // subtrees dealt to `nshards` shards plus a "top" (their common ancestors) factorised redundantly
  // by every shard after one all-reduce of the top fronts' external contributions.
  int nshards = 1;
  int shard = 0;
  // batched leaf columns (dense-column QPs): single-column leaf fronts with >= lb_min_rows update
  // rows, >= lb_min_count of them under one parent and dense enough, are not factorised one by one:
  // their parent absorbs F -= W D^{-1} W^T in one MFMA SYRK (W = their K columns).  Unsharded only.
  int leaf_batch = 1;
  int lb_min_rows = 128;
  int lb_min_count = 64;
  double lb_min_density = 0.5;
};

struct SymbolicPlan {
  int N = 0;
  int64_t nnzK = 0;                    // entries of the caller's lower CSC
  std::vector<int32_t> perm, pinv;     // perm[k] = original index of pivot k
  // supernodes (fronts), in postorder; columns of s are [first[s], first[s+1])
  int nsuper = 0;
  std::vector<int32_t> first, parent, nrows;
  std::vector<int64_t> row_ptr;        // rows[row_ptr[s] .. row_ptr[s+1]) = R_s (permuted ids)
  std::vector<int32_t> rows;           // first w_s entries = own columns, then sorted below rows
  std::vector<int32_t> child_ptr, child_list;
  std::vector<int64_t> rel_ptr;        // rel[rel_ptr[c] ..) = positions of R_c[w_c:] in R_parent
  std::vector<int32_t> rel;
  std::vector<int64_t> asm_ptr;        // per front: original entries (src nz index, local offset)
  std::vector<int64_t> asm_src;
  std::vector<int64_t> asm_dst;        // col_local * r + row_local
  std::vector<int32_t> level;          // height of the front in the supernodal tree
  std::vector<int32_t> level_ptr, level_list;
  int nlevels = 0;
  // storage layout (doubles)
  std::vector<int64_t> l_off;          // L panel (r x w, col-major, ld r); big fronts: whole F
  std::vector<int64_t> u_off;          // update block (ld u_ld)
  std::vector<int32_t> u_ld;
  std::vector<int64_t> uvec_off;       // solve update vector (r - w)
  std::vector<uint8_t> is_big;
  // assembly plan (see symbolic.cpp step 10): every big front and every small front with children
  // is assembled tile by tile (64x64 lower tiles).  The sources of each tile entry (original K
  // entries, then the small children's update entries, fixed order) are cut into chunks of at most
  // kChunk consecutive sources; chunk sums are formed by a flat kernel, then each entry sums its
  // chunks in order (deterministic, no atomics).  Big children (update blocks > kGatherMax rows)
  // are added per tile from their row/column ranges.
  static constexpr int kGatherMax = 128;
  static constexpr int kChunk = 8;
  static constexpr int32_t kAccumulate = INT32_MIN;  // tij flag: F += tile (else F = tile)
  struct AsmTile {
    int32_t front, tij;    // tij = ti | tj << 16 (| kAccumulate)
    int32_t bt0, bt1;      // range in bt (5 ints per big-child block: child, b0, b1, a0, a1)
    int64_t gptr, gchk;    // the tile's entry list in g_ptr (-1: none; ne, ne x (pos | chunk << 12), nchk << 12), first chunk
  };
  std::vector<AsmTile> atiles;
  // assembly groups (ranges of atiles / chunks): g in [0, nlevels) = phase-1 levels (this shard's
  // subtree fronts; every front when unsharded), g = nlevels = the top fronts' external assembly
  // (before the all-reduce), g in (nlevels, 2 nlevels] = phase-2 levels (top fronts, F += the
  // contributions of their top children), g = 2 nlevels + 1 = the factorisation-tree pre-assembly
  std::vector<int32_t> atile_lev;      // size 2 nlevels + 3
  std::vector<int64_t> chunk_lev;
  // single-panel big fronts (w <= 64) whose trailing tiles are assembled and updated by ONE launch
  // after the panel factorisation (k_asm_update): per phase-1 level, the group's tiles are
  // [atile_lev, atile_fz0) plain, [atile_fz0, atile_fz1) the fused fronts' column block 0,
  // [atile_fz1, atile_lev + 1) their other tiles
  std::vector<uint8_t> fused;
  std::vector<int32_t> atile_fz0, atile_fz1;
  std::vector<int32_t> g_ptr, bt;
  hvec<int64_t> g_chunk;               // chunk c = sources [g_chunk[c], g_chunk[c+1])
  hvec<int64_t> g_src;                 // >= 0: arena index; < 0: ~(index into caller's values)
  std::vector<int64_t> fs_off;         // small fronts with children, tree fronts: r x r scratch (else -1)
  static constexpr int kFactTreeMax = 192;
  // medium tree fronts (kFactTreeMax < r <= kFactTreeMedMax): factorised by k_fact_tree in HBM, one
  // 64-column panel in LDS at a time (fact_med_front); big-front storage, pre-assembled in the arena
  static constexpr int kFactTreeMedMax = 256;
  static constexpr int kFoldThreads = 512;  // threads of k_fact_tree: product-list chunks per batch
  static constexpr int kFactTreeFanIn = 8;
  std::vector<uint8_t> ftree;          // factorisation-tree fronts (k_fact_tree)
  std::vector<int32_t> ft_order;       // their ticket order (level by level, longest tail first)
  // leaf folding (tree fronts whose pre-leaf children are all micro leaves: w <= 2, r <= 32): the
  // front factorises its micro leaves in LDS and subtracts their rank-1/2 updates through
  // destination-sorted product lists, instead of k_micro_factor writing update blocks to HBM and
  // the gather pre-assembly summing them.  Leaf rows are flattened per front in child order (ab_*);
  // the leaves are cut into batches whose rows fit LDS beside the front.  Per batch the products
  // (F(i, j) -= l(q1) . p(q2) over the two leaf columns, p = l d) are sorted by LDS destination
  // (leaf order within one destination) and cut into kFoldThreads chunks of equal length, a
  // destination run split where a cut falls (thread t walks chunk t; entry k of chunk t at
  // fold_poff + kFoldThreads k + t, so each load instruction is coalesced).  One 32-bit word per
  // entry: q1 | q2 << 12 | dd << 24 | run end << 31 — batch-local rows (12 bits; kFoldPad as q1: no
  // product) and the step dd of the thread's running destination (from fold_chead's base; a step
  // beyond 127 takes kFoldPad entries).  A run's sum is subtracted at its last entry in the chunk; the
  // first run of a chunk that continues its left neighbour's run is parked in LDS instead and added
  // after the products, left to right (every destination: one atomic writer + a fixed-order tail).
  // r3: cutting only at destination boundaries padded the chunks to the longest run (2x the products
  // at ex10's level-1/2 fronts) and 2 words per entry carried the destination of every product.
  static constexpr int64_t kFactTreeLdsMax = 150 * 1024;  // dynamic LDS of k_fact_tree
  static constexpr int64_t kFoldLdsMax = 148 * 1024;      // fold front + leaf rows (k_fact_tree's
                                                          // static LDS is ~10.4 KB of the CU's 160 KB)
  static constexpr int kFoldRowBytes = 36;                // LDS per leaf row: (l0, l1), (l0 d0, l1 d1), leaf
  static constexpr int kFoldLeafBytes = 48;               // LDS per leaf: d0, d1, f10, L offset, row0, w | rc
  static constexpr uint32_t kFoldRunEnd = 1u << 31;       // entry: last product of its run (in the chunk)
  static constexpr uint32_t kFoldPad = 0xfffu;            // q1 of an entry without a product
  static constexpr int kFoldLeavesMax = 2 * kFoldThreads;  // leaves per batch: fold_leaves' two table registers per thread
  static constexpr int kFoldRowsMax = 4095;               // leaf rows per batch: 12-bit indices below kFoldPad
  static constexpr uint32_t kFoldCont = 1u << 31;         // fold_chead: the chunk's first run continues
  static constexpr int kFoldMaxBatches = 32;              // leaf batches per folding front (LDS table)
  std::vector<uint8_t> absorb;        // front folds its micro leaves
  std::vector<uint8_t> fold_pk;       // fold front stored packed in LDS (to leave room for the leaf rows)
  std::vector<int32_t> mc_ptr, mc_list;  // per front: its folded micro leaves (child order)
  std::vector<int64_t> ab_first;      // per folded leaf: first flat row (rows of front s are contiguous)
  std::vector<int32_t> ab_src0, ab_src1, ab_k;  // per flat row: caller's K index of columns 0 / 1, leaf
  std::vector<int32_t> ab_f0, ab_wrc;  // per folded leaf: first pivot, w | rc << 8 (l_off: LDLSolver)
  std::vector<int32_t> fold_bptr;     // per front: its batches [fold_bptr[s], fold_bptr[s + 1])
  std::vector<int32_t> fold_bat;      // per batch: first leaf index (into mc_list); + end sentinel
  std::vector<int64_t> fold_row0;     // per batch: its first flat leaf row (ab_first of fold_bat); + sentinel
  std::vector<int64_t> fold_poff;     // per batch: first product entry
  std::vector<int32_t> fold_plen;     // per batch: entries per chunk
  std::vector<uint32_t> fold_chead;   // per batch x kFoldThreads: base destination | kFoldCont
  std::vector<int32_t> fold_rmax, fold_lmax;  // per front: largest batch (rows, leaves): its LDS carve
  std::vector<uint32_t> fold_prod;    // one word per entry (above)
  int64_t fs_size = 0;
  // forward-solve gather: for every front row, the children's update-vector entries in child order
  std::vector<int64_t> sv_ptr, sv_src;  // sv_ptr indexed by row_ptr[s] + i
  int64_t arena_size = 0, uvec_size = 0;
  // sharding (nshards > 1): owner[s] = -1 for top fronts (all shards), else the owning shard
  int nshards = 1, shard = 0;
  std::vector<int32_t> owner;
  int64_t top_lo = 0, top_hi = 0;      // arena range of the top fronts (F, full r x r); followed by
                                       // 4 * nshards status slots (fail pivot, +, -, 0 counts)
  std::vector<int64_t> xoff;           // top front -> offset of its rows in the solve exchange vector
  int64_t xlen = 0;                    // sum of the top fronts' orders
  std::vector<int64_t> sx_ptr, sx_src; // top rows (xoff[s] + i): this shard's subtree-root updates
  double top_cost = 0, shard_cost_max = 0, shard_cost_sum = 0;  // partition statistics
  // batched leaf columns: group g = members lb_mem[mem_off .. mem_off + n) (pivot columns, permuted
  // ids) under front `parent`; W (m x n, col-major, ld m) holds their K columns on the rows
  // gpos[gpos_off .. + m) of the parent (sorted local rows); the group's forward update vector lives
  // at uvec[uvec_off ..) and is gathered by the parent like a child's.
  struct LBGroup {
    int32_t parent, m, n, pad;
    int64_t w_off, mem_off, gpos_off, uvec_off;
  };
  std::vector<LBGroup> lb;
  std::vector<int32_t> lb_of;          // per front: group id, -1 if not a member
  std::vector<int32_t> lb_mem;         // member pivot columns
  std::vector<int64_t> lb_cs, lb_ce;   // member j: its entries are the caller's CSC entries [cs, ce)
  std::vector<int64_t> lb_wbase;       // member j: lb_wrow[wbase + (e - cs)] = W row of entry e (-1: diagonal)
  std::vector<int32_t> lb_wrow;
  std::vector<int32_t> lb_gpos;
  int64_t lb_wsize = 0;
  bool mine(int s) const { return owner.empty() || owner[s] == shard; }
  bool top(int s) const { return !owner.empty() && owner[s] < 0; }
  // SURVEY 8(d)'s algorithmic counts per pivot column (permuted ids): nnz of L's column (diagonal
  // included) and of the caller's K in that pivot column (lower triangle in pivot order, diagonal
  // included) -- B_fact = sum 8 colcnt + 12 kcol, B_solve = 2 x 8 sum colcnt
  std::vector<int32_t> colcnt, kcol;
  // statistics
  int64_t nnzL = 0;          // exact nnz(L) incl. diagonal (column counts)
  int64_t nnzL_super = 0;    // stored lower-trapezoid entries incl. relaxed zeros
  double flops = 0;          // sum_j (c_j - 1)(c_j + 2) over stored supernodal columns
  double order_flops_amd = 0, order_flops_nd = 0;  // candidates evaluated by ordering 4 (auto)
  int max_front = 0, nbig = 0;
};

// Analyse the symmetric matrix given by its lower-triangular CSC pattern (0-based, entries with
// row >= col, unique).  Throws madipm::Error on invalid input.
// Host threads of the O(nnz) analysis / construction passes (MADIPM_ANALYSIS_THREADS, default the
// hardware threads, at most 16)
int analysis_threads();

void symbolic_analyze(int N, const int64_t* colptr, const int32_t* rowval, const SymbolicOptions& opt,
                      const int32_t* user_perm, SymbolicPlan& plan);

}  // namespace madipm
