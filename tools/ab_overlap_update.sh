set -e
for i in 1 2; do
  for v in 0 1; do
    VELES_AMD_OVERLAP_UPDATE=$v timeout -k 10 240 python bench.py --steps 40 --warmup 5 > gpurun_out/b_upd_${v}_$i.log 2>&1
    echo "upd=$v run=$i $(grep -o '"value": [0-9.]*' gpurun_out/b_upd_${v}_$i.log)"
  done
done
