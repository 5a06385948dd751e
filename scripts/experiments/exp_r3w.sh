# r3 s2: the C5 FFN down-projection (M = 832, N = 1024, K = 4096, split-K partial) through the 64 x 128
# tile at split 2 / 4 / 8 against the 256 x 256 tile at split 8 (the current choice)
export TMPDIR=/tmp
U=spittle_amd/ubench
for ks in 2 4 8; do timeout -k 5 60 $U gemm 832 1024 4096 8 2 $ks || exit 1; done
