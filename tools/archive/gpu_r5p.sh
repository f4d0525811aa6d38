# round 5: host enqueue time of the benched iteration vs its completion time (4096 and 512 walkers)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python tools/host_probe.py 4096 20 2>&1 | grep -v amdgpu.ids
timeout -k 10 120 python tools/host_probe.py 512 20 2>&1 | grep -v amdgpu.ids
