# A/B of the L.U kernel between builds in abl/libapm_<v>.so (development): tools/ugemm_bench.py per
# build, two alternations; the checksum line shows whether the builds agree bit for bit.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for rep in 1 2; do
  for v in "$@"; do
    echo "== $v"
    APM_LIB=abl/libapm_$v.so timeout -k 10 120 python3 -u tools/ugemm_bench.py --batches ${UB_BATCHES:-1,4,8,21,64} || exit $?
  done
done
