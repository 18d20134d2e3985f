# EXPERIMENT: triangle records padded 48 -> 64 B (lib_t64): the traversal's sensitivity to triangle bytes, beside round 5's 80 -> 128-B nodes (+15 %); interleaved C4 A/B and FETCH/WRITE counter passes of both (serial frames)
set -o pipefail
mkdir -p gpurun_out/r06_c
export TMPDIR=/tmp
T64=ARK_DDGI_LIB=arkoserenderer_amd/lib_t64/libark_ddgi.so
bash tools/ab_bench.sh r06_c_ab $T64 - $T64 - $T64 - || exit 1
bash tools/prof_ab.sh r06_c_pmc --pmc - $T64 || exit 1
