# Effective shader clock of the encoder kernels: GRBM_GUI_ACTIVE (summed over the 8 XCDs) / 8 /
# kernel duration (MI355X_MICROARCH "DVFS give-back"), one --pmc pass with the kernel trace
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/clk
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d gpurun_out/clk -o run -- python3 scripts/probe_kernels.py enc_attn enc_fc1_gemm > gpurun_out/clk.log 2>&1 || { echo "pmc pass failed"; tail -5 gpurun_out/clk.log; exit 1; }
python3 scripts/pmc_clock_parse.py > gpurun_out/clk_summary.txt; cat gpurun_out/clk_summary.txt
