# r3 s2: the Parakeet offline shapes (8 x 30 s: M = 3000) through every tile: which one wins where the
# 256 x 256 tile gives under one workgroup per CU (q/k/v 144, pw1 96, FFN up 192 workgroups)
export TMPDIR=/tmp
U=spittle_amd/ubench
for cfg in "3000 4096 1024 5 2" "3000 3072 1024 0 2" "3000 2048 1024 0 2" "3000 1024 4096 8 2 1" "3000 1024 4096 8 2 2" "3000 1024 4096 8 2 4" "3000 1024 1024 8 2 1" "3000 1024 1024 8 2 2" "3000 1024 1024 8 2 4"; do
  timeout -k 5 60 $U gemm $cfg || exit 1
done
