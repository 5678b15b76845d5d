# determinism soak: the stationary 64-chain theta-call + u-call, APM_OVERLAP_K alternating over
# 12 contexts x 4 calls with HIP-event profiling from the second call (tools/det_check.py)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05det; mkdir -p $O
timeout -k 10 800 python -u tools/det_check.py APM_OVERLAP_K 1 0 1 0 1 0 1 0 1 0 1 0 --calls 4 --prof 2>&1 | tee $O/det_soak.txt
