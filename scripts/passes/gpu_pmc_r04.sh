#!/bin/bash
# Round-4 HBM traffic passes (share blocks from memory.share_block) (MI355X_MICROARCH.md §HBM): separate rocprofv3
# --pmc passes (FETCH_SIZE; WRITE_SIZE; TCC_EA0_RDREQ_sum + TCC_EA0_WRREQ_sum),
# kernel trace only, over scripts/prof_kernels.py (split, reconstruct, fused
# MT draw + split, mask row at 2^24).  Each pass has its own time limit.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-pmc_r04}
mkdir -p $O
export TMPDIR=/tmp
rc=0
cd /tmp
for pass in "pmc_fetch FETCH_SIZE" "pmc_write WRITE_SIZE" "pmc_req TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  set -- $pass
  name=$1; shift
  [ $rc = 0 ] || break
  echo "== $name"
  timeout -s KILL 150 rocprofv3 --pmc "$@" --kernel-trace -d /tmp/$name -o run --output-format csv -- python3 "$R/scripts/prof_kernels.py" > "$R/$O/$name.log" 2>&1 || rc=$?
  find /tmp/$name -name "*counter_collection.csv" -exec cp {} "$R/$O/$name.csv" \;
done
cd "$R"
if [ $rc = 0 ]; then
  python3 scripts/pmc_summary.py $O $O/pmc_traffic.json 24 "${SRC:-round 4}" > $O/summary.txt 2>&1 || rc=$?
  grep -E '"(split|reconstruct|fused_draw_split|mask_accumulate)"|traffic_over' $O/pmc_traffic.json
fi
echo "== rc $rc"
exit $rc
