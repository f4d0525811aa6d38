set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 120 ./tools/valu_rate > gpurun_out/valu_rate.txt 2>&1; cat gpurun_out/valu_rate.txt | grep -v amdgpu.ids
