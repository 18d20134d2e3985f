# end of round 6, the final tree (lib 5ebc5676): the GPU suite, smoke, the driver bench command
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_check.sh r06_final7 --no-prof || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06_final7/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r06_final7/smoke.log; exit 1; }
tail -2 gpurun_out/r06_final7/smoke.log
echo done
