mkdir -p gpurun_out
for v in "c1:copy" "c2:copy" "k1:kernel" "k2:kernel" "k3:kernel" "n1:none" "n2:none" "n3:none"; do
  n=${v%%:*}; m=${v#*:}
  MPA_GRAPH_COPY=$m timeout -k 10 300 python bench.py --steps 80 --warmup 3 --static-data --batch 128 --graph on > gpurun_out/race_$n.log 2>&1 || exit $?
  echo "$n $m $(grep -o '"mean_loss": [^}]*' gpurun_out/race_$n.log)"
done
