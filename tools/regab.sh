set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for v in "A:COA_REGISTER_CUS=128 COA_BUILD_BLOCKS=1024" "B:COA_REGISTER_CUS=0 COA_BUILD_BLOCKS=128" "C:COA_REGISTER_CUS=0 COA_BUILD_BLOCKS=0" "D:COA_REGISTER_CUS=128 COA_BUILD_BLOCKS=0" "E:COA_REGISTER_CUS=128 COA_BUILD_BLOCKS=1024 COA_QUEUE_DIGEST_SLOTS=1 COA_QUEUE_SLOTS=2"; do
  name=${v%%:*}; assign=${v#*:}
  env $assign timeout -k 10 120 python -u tools/register_probe.py 5000 3 2 > gpurun_out/regab_$name.json 2> gpurun_out/regab_$name.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/regab_$name.json'));print('$name', '$assign', d['p99_ms_during'], d['max_ms_during'], d['p99_ms_outside'], d['registrations_s'])"
done
