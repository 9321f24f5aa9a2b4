cd "${GRAFT_REPO_ROOT}" && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 5 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_sign_sha.py tests/test_gpu_sanitize.py > gpurun_out/t_sha.log 2>&1; tail -2 gpurun_out/t_sha.log
grep -q passed gpurun_out/t_sha.log && ! grep -q failed gpurun_out/t_sha.log || exit 1
for rep in 1 2; do
  for kv in new=xrpl-coa-prototype_amd/lib/libcoa_verify.so old=build/ab/libcoa_verify_prev.so; do
    name=${kv%%=*}; lib=${kv#*=}
    COA_VERIFY_LIB=$PWD/$lib timeout -k 10 240 python bench.py --no-cpu-baseline --steps 5 --warmup 1 --c3-certs 1000 \
      > gpurun_out/abs_$name.json 2>gpurun_out/abs_$name.err || { tail -5 gpurun_out/abs_$name.err; exit 1; }
    python -c "
import json;d=json.load(open('gpurun_out/abs_$name.json'))['secondary']['c4_sha512']
print('$name', {k:v for k,v in d.items() if k.startswith('batches')})"
  done
done
