#!/bin/bash
# Round-3 pass r: the ChaCha20 split under sustained load (scripts/prng_heat.py),
# with rocm-smi's clock / power readout (read only) before and after.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r03r}
mkdir -p $O
rc=0
(rocm-smi --showclocks --showpower --showtemp > $O/smi_before.txt 2>&1 || true)
timeout -k 10 200 python scripts/prng_heat.py > $O/prng_heat.json 2> $O/prng_heat.err || rc=$?
(rocm-smi --showclocks --showpower --showtemp > $O/smi_after.txt 2>&1 || true)
cat $O/prng_heat.json; grep -iE "sclk|power|temp" $O/smi_after.txt | head -12
echo "== rc $rc"
exit $rc
