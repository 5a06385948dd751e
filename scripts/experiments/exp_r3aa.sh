# r3 s2: Parakeet relative attention with the key tiles split over 4 waves (merged through LDS) vs
# one wave (SPT_PK_ATTN_NW=1): parity, then the Parakeet lines
export TMPDIR=/tmp
mkdir -p gpurun_out
true
true
for nw in 2 1; do
  SPT_PK_ATTN_NW=$nw timeout -k 10 300 python3 bench.py --parakeet-only --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r3aa_pk$nw.log 2>&1 || { tail -5 gpurun_out/r3aa_pk$nw.log; exit 1; }
done
echo bench done
