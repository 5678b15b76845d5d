set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for b in tools/upd64_a*.bin; do timeout -k 5 60 $b; done > gpurun_out/u64.log 2>&1
cat gpurun_out/u64.log
