# determinism soak of the default path: the stationary 64-chain theta-call + u-call, 8 contexts x
# 8 calls each, HIP-event profiling on from the second call of each context (tools/det_check.py)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05det; mkdir -p $O
timeout -k 10 600 python -u tools/det_check.py APM_OVERLAP_K 1 1 1 1 1 1 1 1 --calls 8 --prof 2>&1 | tee $O/det_final.txt
