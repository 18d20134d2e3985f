# bench.py's Z-slab rank path rehearsed on one GPU (ARK_BENCH_REHEARSAL=1: gloo, every rank on cuda:0, host-staged all-gather): 2 and 4 ranks, whole grid and a 2,048-probe window
set -o pipefail
OUT=gpurun_out/r06_t
mkdir -p $OUT
export TMPDIR=/tmp
export ARK_BENCH_REHEARSAL=1
for n in 2 4; do
  timeout -k 10 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2961$n bench.py --gpus $n --steps 5 --warmup 2 > $OUT/rehearsal_$n.log 2>&1 || { echo "rehearsal $n failed rc=$?"; tail -30 $OUT/rehearsal_$n.log; exit 1; }
  tail -1 $OUT/rehearsal_$n.log | cut -c1-400
done
timeout -k 10 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29619 bench.py --gpus 2 --steps 20 --warmup 3 --probe-updates 2048 > $OUT/rehearsal_2_k2048.log 2>&1 || { echo "rehearsal k2048 failed rc=$?"; tail -30 $OUT/rehearsal_2_k2048.log; exit 1; }
tail -1 $OUT/rehearsal_2_k2048.log | cut -c1-400
echo done
