# Counter passes of the Newton factorisation's kernels alone (round-5 verdict item 4): two
# stationary 64-chain theta-calls (tools/time_theta.py on the long-chain record's states) with
# APM_POST32=0, so that every k_chol_update32_t128 dispatch is a Newton trailing update (the
# posterior bottom block, which shares that kernel, then runs in fp64). One rocprofv3 run per
# pass, each under its own time limit; summaries by tools/pmc_kernels.py, raw CSVs deleted.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pmc_newton; mkdir -p $O
export APM_POST32=0
CMD="python3 tools/time_theta.py --batch 64 --reps 2 --no-prof --theta-file profiles/r04_stationary_thetas.npy"
timeout -s KILL 60 rocprofv3 -L > $O/counters_list.txt 2>&1 || true
run() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $O/$name -o run -- $CMD > $O/$name.log 2>&1
  local rc=$?
  echo "pass $name: exit $rc"
  return $rc
}
run mfma SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE || exit $?
run insts SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES || exit $?
run waits SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU || exit $?
run fetch FETCH_SIZE || exit $?
run write WRITE_SIZE TCC_HIT_sum TCC_MISS_sum || exit $?
F=""
for p in mfma insts waits fetch write; do
  c=$(find $O/$p -name '*counter_collection.csv' | head -1)
  [ -n "$c" ] && F="$F $c"
done
python3 tools/pmc_kernels.py --match k_chol_update32_t128 --match k_chol_update32_q256 --match k_panel_inv_gemm32 --match k_zinv --match k_chol_panel_df32 --match k_trsv32_mw --match k_symv_part --match k_chol_update_t128 $F --json $O/summary.json > $O/summary.txt 2>&1
find $O -name '*.csv' -delete
echo done
