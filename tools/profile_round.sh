# Round profile of the default bench (3 timed steps): kernel trace + stats, then separate PMC passes
# (FETCH_SIZE; WRITE_SIZE; SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE) of the same command; the
# timed-window summary (tools/prof_window.py) is written on the box and the raw per-dispatch CSVs
# are deleted (gpurun copies back <= 64 MiB). The summary records bench.csrc_sha16() of the profiled
# sources and profiles/BUILD_COMMIT (written by `git describe --always --dirty` before the call),
# so bench.py can tell whether a committed PMC pass describes the build it runs.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/prof_round
mkdir -p $O
CMD="python3 bench.py --steps 3 --warmup 5 --cpu-baseline 0 --parity 0 --ess-min 0 --ess-burn 0"
SHA=$(python3 -c "import bench; print(bench.csrc_sha16())")
COMMIT=$(cat profiles/BUILD_COMMIT 2>/dev/null || echo unknown)
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- $CMD > $O.trace.json 2> $O.trace.err
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch -o run -- $CMD > $O.fetch.json 2> $O.fetch.err
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/write -o run -- $CMD > $O.write.json 2> $O.write.err
timeout -k 10 400 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/mfma -o run -- $CMD > $O.mfma.json 2> $O.mfma.err
T=$(find $O/trace -name '*kernel_trace.csv' | head -1)
F=$(find $O/fetch -name '*counter_collection.csv' | head -1)
W=$(find $O/write -name '*counter_collection.csv' | head -1)
M=$(find $O/mfma -name '*counter_collection.csv' | head -1)
python3 tools/prof_window.py "$T" --fetch "$F" --write "$W" --mfma "$M" --out $O/window.json \
    --csrc-sha16 "$SHA" --commit "$COMMIT" > $O/window.txt
python3 tools/idle_gaps.py "$T" > $O/idle_gaps.txt
find $O -name '*kernel_trace.csv' -delete
find $O -name '*counter_collection.csv' -delete
du -sh $O
