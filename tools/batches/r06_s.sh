# EXPERIMENT whole-grid pipelined traversal at 3/4/5 workgroups per CU (g3/g4/g5) against the full grid (shipped), C4, interleaved twice
set -o pipefail
G3=ARK_DDGI_LIB=arkoserenderer_amd/lib_g3/libark_ddgi.so
G4=ARK_DDGI_LIB=arkoserenderer_amd/lib_g4/libark_ddgi.so
G5=ARK_DDGI_LIB=arkoserenderer_amd/lib_g5/libark_ddgi.so
bash tools/ab_bench.sh r06_s --no-configs --steps 20 -- - $G3 $G4 $G5 - $G3 $G4 $G5 || exit 1
echo done
