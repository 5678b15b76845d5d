# the bench under the driver's invocation (after the round profile of the same build is committed,
# so that its pmc_provenance is not stale)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05b; mkdir -p $O
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || { echo "bench failed"; tail -20 $O/bench20.err; exit 1; }
tail -c 300 $O/bench20.json
