# round 6: small-batch walker launch on two waves per walker (F1 || F2, AIQMC_WALK_SPLIT=1, the default for
# B <= 8 x CUs) against one wave (AIQMC_WALK_SPLIT=0): N2 positions / E_L bitwise, then the loop at 512 / 1024 /
# 2048 walkers (the per-rank batches of 8 / 4 / 2 GPUs), interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for v in 0 1; do
  AIQMC_WALK_SPLIT=$v timeout -k 10 120 python tools/pos_dump.py gpurun_out/ab/pos_ws$v.npy N2 ${POS_WALKERS:-512} > /dev/null 2>&1 || { echo "pos_dump $v FAILED"; exit 1; }
done
python3 -c "
import numpy as np
a, b = np.load('gpurun_out/ab/pos_ws0.npy'), np.load('gpurun_out/ab/pos_ws1.npy')
print('split vs one wave: bitwise equal', np.array_equal(a, b), 'max |diff|', float(np.max(np.abs(a - b))))"
for rep in 1 2; do
  for B in 512 1024 2048; do
    for v in 0 1; do
      r=$(AIQMC_WALK_SPLIT=$v timeout -k 10 120 python tools/mc_loop.py 20 N2 $B 2>&1 | grep -v amdgpu.ids) || { echo "loop $v $B FAILED"; exit 1; }
      echo "split=$v rep$rep $r"
    done
  done
done
