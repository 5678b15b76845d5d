# Cohort overlap at stationarity: the bench workload as 1 or 2 contexts of 64 / 32 chains, each
# driven by its own host thread, started from the long-chain record's states.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05c; mkdir -p $O
timeout -k 10 400 python -u tools/cohort_bench.py --cohorts 1 2 --steps 12 --warmup 3 --stationary profiles/r04_stationary_thetas.npy > $O/cohorts.txt 2>&1
rc=$?; cat $O/cohorts.txt | grep -v amdgpu.ids; exit $rc
