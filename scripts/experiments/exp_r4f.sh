# r4f: test_beam_search[5-20-91] failed after the straight-line attention schedule; the same case
# under the round-start build (DIAG_LIB) and the cross-attention variants
export TMPDIR=/tmp
mkdir -p gpurun_out
L=spittle_amd/libspittle_hip_head.so
OR=1 DIAG_LIB=$L timeout -k 10 200 python3 -u scripts/experiments/diag_beam.py > gpurun_out/r4f_0.log 2>&1 || { tail -20 gpurun_out/r4f_0.log; exit 1; }
timeout -k 10 120 python3 -u scripts/experiments/diag_beam.py > gpurun_out/r4f_1.log 2>&1 || { tail -20 gpurun_out/r4f_1.log; exit 1; }
SPT_XATTN_VW=0 timeout -k 10 120 python3 -u scripts/experiments/diag_beam.py > gpurun_out/r4f_2.log 2>&1 || { tail -20 gpurun_out/r4f_2.log; exit 1; }
SPT_XATTN_VW=2 timeout -k 10 120 python3 -u scripts/experiments/diag_beam.py > gpurun_out/r4f_3.log 2>&1 || { tail -20 gpurun_out/r4f_3.log; exit 1; }
SPT_NO_WINDOW_SHARE=1 timeout -k 10 120 python3 -u scripts/experiments/diag_beam.py > gpurun_out/r4f_4.log 2>&1 || { tail -20 gpurun_out/r4f_4.log; exit 1; }
SPT_XATTN_VW=0 DIAG_LIB=$L timeout -k 10 120 python3 -u scripts/experiments/diag_beam.py > gpurun_out/r4f_5.log 2>&1 || { tail -20 gpurun_out/r4f_5.log; exit 1; }
grep -h -E "^(env|oracle)" gpurun_out/r4f_*.log
