# HIP runtime knobs for launch latency inside the decode graphs (bench A/B, environment only)
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {
  env "$@" timeout -k 10 300 python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-app-latency --no-parakeet --no-probe > gpurun_out/g9.log 2>&1 || { echo "bench failed: $*"; tail -5 gpurun_out/g9.log; exit 1; }
  echo "$* $(tail -1 gpurun_out/g9.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["phases_ms"]["decode_ms"], d["rooflines"]["decode_pass"]["ms_per_pass"])')"
}
run X=0
run HIP_FORCE_DEV_KERNARG=1
run HIP_FORCE_DEV_KERNARG=0
run DEBUG_CLR_GRAPH_PACKET_CAPTURE=1
run DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
run X=0
