# the sun's shadow-ray structure, world BVHs vs the light-space BVH, interleaved in one process, and counter passes of both
set -o pipefail
OUT=gpurun_out/r06_e
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/sun_ab.py --reps 5 > $OUT/sun_ab.log 2>&1 || { echo "sun_ab failed"; tail -20 $OUT/sun_ab.log; exit 1; }
tail -1 $OUT/sun_ab.log | cut -c1-1500
bash tools/prof_ab.sh r06_e_sunpmc --pmc "--sun-bvh world" "--sun-bvh light" || exit 1
echo done2
