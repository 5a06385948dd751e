# interleaved-tile encoder attention (SPT_ATTN_SUM=5) vs the optimistic kernel (3): output diff, probes
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 3 5 3 5; do
SPT_ATTN_SUM=$v timeout -k 10 120 python3 scripts/enc_dump.py s$v > gpurun_out/g8_$v.log 2>&1 || { tail -5 gpurun_out/g8_$v.log; exit 1; }
echo "sum=$v $(tail -1 gpurun_out/g8_$v.log)"
done
python3 -c "import numpy as np; a=np.load('gpurun_out/enc_s3.npy'); b=np.load('gpurun_out/enc_s5.npy'); print('bitwise', np.array_equal(a,b), 'rel L2', float(np.linalg.norm(a-b)/np.linalg.norm(a)))"
