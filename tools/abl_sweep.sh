set -e
for a in 0 1 2 4 3 7; do
  echo "ABL=$a"
  ESP_GEMM_ABL=$a timeout -k 10 100 python tools/gemm_ksweep.py 23936 1024
done
