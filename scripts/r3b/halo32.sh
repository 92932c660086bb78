#!/bin/bash
# 32-wide halo forward / zero-padded halo wgrad / split-K finalize: tests, then the zoo conv tables
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "halo or splitk or autotune" > $O/t_halo32.log 2>&1
rc=$?; tail -3 $O/t_halo32.log; [ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" $O/t_halo32.log | head -20; exit $rc; }
timeout -k 10 300 python tools/bench_zoo_convs.py densenet 256 5 > $O/zoo_densenet2.txt 2>&1 || { tail -5 $O/zoo_densenet2.txt; exit 1; }
head -8 $O/zoo_densenet2.txt
timeout -k 10 300 python tools/bench_zoo_convs.py inception 256 5 > $O/zoo_inception2.txt 2>&1 || { tail -5 $O/zoo_inception2.txt; exit 1; }
head -6 $O/zoo_inception2.txt
timeout -k 10 300 python bench.py --model densenet --batch 256 --steps 10 --warmup 3 --small-batch 0 > $O/b_dn.json 2> $O/b_dn.err || { tail -5 $O/b_dn.err; exit 1; }
cat $O/b_dn.json
timeout -k 10 300 python bench.py --model inception --image-size 299 --batch 256 --steps 10 --warmup 3 --small-batch 0 > $O/b_inc.json 2> $O/b_inc.err || { tail -5 $O/b_inc.err; exit 1; }
cat $O/b_inc.json
