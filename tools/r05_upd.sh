# Standalone timing of the Newton trailing update for every outer panel (tools/upd32_bench.cpp,
# built on the box), e.g. bash tools/r05_upd.sh [-DVARIANT=...]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05c; mkdir -p $O
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -Wno-unused-value -Wno-unused-result $1 -x hip tools/upd32_bench.cpp -o /tmp/upd32 || exit 1
for K in 0 1 2 3 4 5 6; do timeout -k 5 60 /tmp/upd32 64 $K 10 || exit $?; done | tee $O/upd32$2.txt
