#!/bin/bash
# Round-5 pass t: the headline step timed with fence-free HIP events
# (bench.py --events nofence, TimingEvent) against torch.cuda.Event
# (--events torch), at 2^21 (the N = 8 shard) and 2^24, alternating processes.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r05t}
mkdir -p $O
export TMPDIR=/tmp
rc=0
for r in 1 2; do
  for L in 21 24; do
    for ev in nofence torch; do
      echo "== $L $ev $r" && timeout -k 10 240 python bench.py --log2n $L --events $ev --rows 0 --config4 0 --config5 0 --cold 0 --cpu-budget 0 > $O/b_${L}_${ev}_$r.json 2> $O/b_${L}_${ev}_$r.err || { rc=$?; tail -3 $O/b_${L}_${ev}_$r.err; break 3; }
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(d['value']/1e9, d['ms_per_step'], r['avg_launch_ms'], r['frac'], d['kernels']['reconstruct_ms'])" $O/b_${L}_${ev}_$r.json
    done
  done
done
echo "== rc $rc"
exit $rc
