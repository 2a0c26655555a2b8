# A/B of the 512-thread 128x128 fp32 conv tile (4) against the 128x64 stream-K / 64x64 forms
set -e
mkdir -p gpurun_out
for s in ${SHAPES:-l1c1 l1c2 l1c3 ds1 l2c1 l2c2s l2c2 l2c3 ds2 l3c1 l3c2s l3c2 l3c3 ds3 l4c1 l4c2s l4c2 l4c3 ds4}; do
  for t in ${TILES:-0 2 3 4}; do echo "== $s tile $t" >> gpurun_out/w8_ab.log; timeout -k 10 60 python tools/gemm_one.py --shape $s --tile $t >> gpurun_out/w8_ab.log 2>&1; done
done
