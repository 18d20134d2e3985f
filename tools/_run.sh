set -o pipefail
L=$PWD/arkoserenderer_amd/lib
ARK_DDGI_LIB=$L/libark_ddgi_mix.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bake.py tests/test_gpu_sharded.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r01s3_pt3.log 2>&1; rc=$?; tail -2 gpurun_out/r01s3_pt3.log; [ $rc -eq 0 ] || { grep -E "assert|Error" gpurun_out/r01s3_pt3.log | head; exit 1; }
bash tools/sweep_env.sh r01s3_mix "ARK_DDGI_LIB=$L/libark_ddgi.so" "ARK_DDGI_LIB=$L/libark_ddgi_mix.so" "ARK_DDGI_LIB=$L/libark_ddgi.so" "ARK_DDGI_LIB=$L/libark_ddgi_mix.so"
