# r3: encoder attention softmax variants (SPT_ATTN_SUM): 3 = optimistic, packed f32 VALU (r2 default);
# 4 = optimistic, scalar f32 FMAs and adds; 5 = optimistic, scalar FMAs, row sums on the MFMA pipe
# (ones . P^T) and the re-base decided from the raw score maximum.  Probe: 20 launches at large-v3
# B = 8 in situ, plus the whole encoder.
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 3 4 5 3 4 5; do
  SPT_ATTN_SUM=$v timeout -k 10 200 python3 scripts/probe_kernels.py enc_attn > gpurun_out/probe_r3d.log 2>&1 || { echo "probe failed: $v"; tail -5 gpurun_out/probe_r3d.log; exit 1; }
  echo "SUM=$v $(tail -1 gpurun_out/probe_r3d.log)"
done
