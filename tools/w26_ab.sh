#!/bin/bash
# Same-box A/B of the radix-2^24 (11 positions, 8.9 GB) against the
# radix-2^26 (10 positions, 32 GB) wide B comb (tools/build_variant.py w26):
# device open + whole-table self test, the C2 line with its single/mid/C3/C1
# sections, alternating REPS times.  One JSON per run under gpurun_out/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
LIBS=${LIBS:-"w24=xrpl-coa-prototype_amd/lib/libcoa_verify.so w26=build/w26/libcoa_verify.so"}
for rep in $(seq ${REPS:-2}); do
  for kv in $LIBS; do
    name=${kv%%=*}; lib=${kv#*=}
    COA_VERIFY_LIB=$PWD/$lib timeout -k 10 120 python - <<'PY' > gpurun_out/w26ab_open_${name}_$rep.txt || exit 1
import time, sys
sys.path.insert(0, "xrpl-coa-prototype_amd")
import coa_crypto as c
t = time.perf_counter(); c.init(1); t1 = time.perf_counter()
bad = c.self_test(0); t2 = time.perf_counter()
print(f"open_s {t1 - t:.3f} self_test_s {t2 - t1:.3f} bad {bad}")
PY
    COA_VERIFY_LIB=$PWD/$lib timeout -k 10 400 python bench.py --no-cpu-baseline --steps 40 \
      --sections verify_single,verify_mid,c3_certificate_verify,c1_certificate_verify \
      > gpurun_out/w26ab_${name}_$rep.json 2>gpurun_out/w26ab_${name}_$rep.err || exit 1
    echo "$name $rep $(cat gpurun_out/w26ab_open_${name}_$rep.txt) $(python -c "import json;d=json.load(open('gpurun_out/w26ab_${name}_$rep.json'));print(d['value'], d['summary'])")"
  done
done
