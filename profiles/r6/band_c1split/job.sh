# band forward conv1 unit split sweep (MNISTX_BAND_C1), kernel alone then the step
set -o pipefail
O=gpurun_out/r6s2/c1split; mkdir -p $O
for c in "13,13,13,13" "12,12,12,13" "11,11,11,16" "10,10,10,19" "12,11,11,15" "13,13,13,13"; do
  MNISTX_BAND_C1=$c timeout -k 10 120 python bench/micro_band.py one 2 65536 > $O/m_$c.txt 2>&1 || { tail -5 $O/m_$c.txt; exit 1; }
  echo "$c $(tail -1 $O/m_$c.txt) $(head -1 $O/m_$c.txt | cut -c1-200)"
done
for i in 1 2; do for c in "13,13,13,13" "11,11,11,16" "10,10,10,19"; do
  MNISTX_BAND_C1=$c timeout -k 10 200 python bench.py > $O/b_${c}_$i.json 2>$O/b.err || { tail -5 $O/b.err; exit 1; }
  echo "bench $c $(grep -o '"ms_per_step": [0-9.]*' $O/b_${c}_$i.json) $(grep -o '"forward": [0-9.]*' $O/b_${c}_$i.json)"
done; done
