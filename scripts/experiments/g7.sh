# Parakeet conv-module vectorisation: parity + Parakeet bench lines
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parakeet.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/g7_tests.log 2>&1
rc=$?; tail -3 gpurun_out/g7_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --parakeet-only --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/g7_pk.json 2> gpurun_out/g7_pk.err || { tail -5 gpurun_out/g7_pk.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/g7_pk.json').read().strip().splitlines()[-1]); pk=d.get('parakeet_v3', d.get('parakeet', d))
print(json.dumps({k: (v.get('rtfx'), v.get('phases_ms'), v.get('encoder_roofline',{}).get('frac')) if isinstance(v, dict) and 'rtfx' in v else v for k, v in pk.items() if k.startswith(('stream','off'))}))"
