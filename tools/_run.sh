set -o pipefail
L=$PWD/arkoserenderer_amd/lib
ARK_DDGI_LIB=$L/libark_ddgi_bl.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bake.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r01s3_pt4.log 2>&1; rc=$?; echo "bl: $(tail -1 gpurun_out/r01s3_pt4.log)"; [ $rc -eq 0 ] || exit 1
bash tools/sweep_env.sh r01s3_bl "ARK_DDGI_LIB=$L/libark_ddgi.so" "ARK_DDGI_LIB=$L/libark_ddgi_bl.so" "ARK_DDGI_LIB=$L/libark_ddgi.so" "ARK_DDGI_LIB=$L/libark_ddgi_bl.so"
