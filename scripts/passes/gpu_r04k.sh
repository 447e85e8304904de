#!/bin/bash
# Round-4 pass k: producer/consumer generation (mt_gen_pc_kernel): MT / fused
# / sharded / config-4 / memory GPU tests on the in-tree library, then
# scripts/msv_ab.py alternating the in-tree library and the one-wave variant
# (lib/ab/libdn_shamir_onewave.so, -DDN_MT_PC=0), then the rocprof kernel
# stats of one msv_ab run per library.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r04k}
mkdir -p $O
export TMPDIR=/tmp
rc=0
echo "== tests" && timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py tests/test_gpu_memory.py -x -q -m gpu -k "${TESTK:-mt or draw or fused or sharded or config4 or digest or memory or block or shares_vec}" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || rc=$?
tail -2 $O/pytest.log
[ $rc -ne 0 ] && { echo "== rc $rc"; grep -E "FAILED|Error" $O/pytest.log | head; exit $rc; }
ab() { if [ "$1" = new ]; then timeout -k 10 200 python scripts/msv_ab.py; else DN_SHAMIR_LIB="$R/delta-node_amd/lib/ab/libdn_shamir_$1.so" timeout -k 10 200 python scripts/msv_ab.py; fi; }
for i in 1 2; do
  for v in new ${VARIANTS:-onewave}; do
    echo "== ab $v $i" && ab $v >> $O/ab_$v.jsonl 2>> $O/ab.err || rc=$?
    [ $rc -ne 0 ] && { echo "== rc $rc"; tail -5 $O/ab.err; exit $rc; }
  done
done
for v in new ${VARIANTS:-onewave}; do cut -c1-420 $O/ab_$v.jsonl; done
for v in ${PROF:-new onewave}; do
  echo "== rocprof $v"
  if [ $v = new ]; then (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pk_$v -o run --output-format csv -- python3 "$R/scripts/msv_ab.py" > "$R/$O/prof_$v.json" 2> "$R/$O/prof_$v.err") || rc=$?
  else (cd /tmp && DN_SHAMIR_LIB="$R/delta-node_amd/lib/ab/libdn_shamir_$v.so" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pk_$v -o run --output-format csv -- python3 "$R/scripts/msv_ab.py" > "$R/$O/prof_$v.json" 2> "$R/$O/prof_$v.err") || rc=$?; fi
  [ $rc -ne 0 ] && { echo "== rc $rc"; tail -3 $O/prof_$v.err; exit $rc; }
  find /tmp/pk_$v -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_$v.csv \;
  grep -E "mt_gen|mt_jump" $O/kernel_stats_$v.csv | cut -d, -f1-4 | cut -c1-160
done
echo "== rc $rc"
exit $rc
