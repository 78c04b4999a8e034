# Placement root-cause probe (dev): event timing of 8 stages, then one
# rocprofv3 PMC pass per counter group, each in its own process (8 fresh
# stages per process; per-stage counters vs per-stage kernel duration).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/place
mkdir -p $O
timeout -k 10 120 python3 tools/placement_pmc.py --rounds 3 --reps 10 --out $O/timing.json > $O/timing.log 2>&1 || exit 1
cat $O/timing.log
pass() {
  local name=$1; shift
  mkdir -p $O/$name
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $O/$name -o run -- python3 tools/placement_pmc.py --rounds 1 --reps 4 --out $O/$name/probe.json > $O/$name/log.txt 2>&1 || return 1
  python3 tools/placement_pmc_summary.py $O/$name | tee $O/$name/summary.txt
}
pass utcl TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_WRITE_REQ_LATENCY_sum || exit 2
pass stall TCC_EA0_WRREQ_STALL_sum TCC_TAG_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE || exit 3
pass dram TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_WRREQ_LEVEL_sum || exit 4
pass utcl2 TCP_TCC_READ_REQ_LATENCY_sum TCP_UTCL1_STALL_INFLIGHT_MAX_sum TCP_UTCL1_SERIALIZATION_STALL_sum TCP_UTCL1_THRASHING_STALL_sum || exit 5
