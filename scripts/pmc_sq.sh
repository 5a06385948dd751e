# SQ counter passes (issue / wait breakdown) over the encoder kernels: one probe run per pass
export TMPDIR=/tmp
mkdir -p gpurun_out
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA"
P2="SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_MISC"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d gpurun_out/sq_$i -o run -- python3 scripts/probe_kernels.py enc_attn enc_fc1_gemm > gpurun_out/sq_$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/sq_$i.log; exit 1; }
done
python3 scripts/pmc_sq_parse.py > gpurun_out/sq_summary.txt; cat gpurun_out/sq_summary.txt
rm -rf gpurun_out/sq_1 gpurun_out/sq_2
