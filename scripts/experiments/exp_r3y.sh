# r3 s2: 64 x 64 GEMM tile (variant 5) against 64 x 128 (4), 128 x 128 (1) and 256 x 256 (2) at the
# C5 shapes and the single-window Whisper shapes; bitwise comparison against the 128 x 128 tile
export TMPDIR=/tmp
U=spittle_amd/ubench
for cfg in "832 4096 1024 5 2" "832 3072 1024 0 2" "832 2048 1024 0 2" "832 1024 4096 8 2 4" "832 1024 4096 8 2 2" "832 1024 1024 8 2 2" "832 1024 1024 8 2 1" "1500 1280 1280 3 1" "1500 1280 5120 3 1" "1500 3840 1280 0 1" "3000 1280 384 2 1"; do
  timeout -k 5 60 $U gemm $cfg || exit 1
done
