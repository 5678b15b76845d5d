# determinism soak of the off-default APM_OVERLAP_K=0 path (chol(K) after the Newton loop, where the
# one 120-nat discrepancy was seen): 8 contexts x 8 calls, HIP-event profiling on from the second call
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05det; mkdir -p $O
timeout -k 10 600 python -u tools/det_check.py APM_OVERLAP_K 0 0 0 0 1 0 0 0 0 --calls 8 --prof 2>&1 | tee $O/det_ovk0.txt
