set -o pipefail
L=$PWD/arkoserenderer_amd/lib
ARK_TRACE_WPE=7 ARK_DDGI_LIB=$L/libark_ddgi_s4.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r01s3_pt4.log 2>&1; rc=$?; echo "s4w7: $(tail -1 gpurun_out/r01s3_pt4.log)"; [ $rc -eq 0 ] || exit 1
bash tools/sweep_env.sh r01s3_occ "ARK_DDGI_LIB=$L/libark_ddgi.so" "ARK_DDGI_LIB=$L/libark_ddgi_s4.so" "ARK_TRACE_WPE=7 ARK_DDGI_LIB=$L/libark_ddgi_s4.so" "ARK_TRACE_WPE=7 ARK_DDGI_LIB=$L/libark_ddgi.so"
