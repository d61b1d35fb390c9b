"""Prints the ROCPROF* / ROCPROFILER* / HSA_TOOLS* environment names a profiler run sets (their values
are not needed): python tools/env_probe.py under rocprofv3 --pmc / --kernel-trace."""
import os
print(sorted(k for k in os.environ if k.startswith(("ROCPROF", "ROCP_", "HSA_TOOLS", "AMD_SERIALIZE", "HIP_LAUNCH"))))
