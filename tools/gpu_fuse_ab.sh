# A/B of hand-off variants of the interval kernel (sweep leg of bench.py), two rounds each
set -o pipefail
tools/gpu_variants.sh pub "a:quantumsimulations_amd/libdse_a.so:" "u0p2:quantumsimulations_amd/libdse_u0p2.so:" "u0p3:quantumsimulations_amd/libdse_u0p3.so:" "u1p3:quantumsimulations_amd/libdse_u1p3.so:"
