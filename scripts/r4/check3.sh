#!/bin/bash
# round 4 call 3: BN link with the unspilled producer-wave BNRED flavour (tests + A/B), PMC
# passes over the b1024 step (where do the halo kernels' cycles go)
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "halo or bnred" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/r4c3_tests.log 2>&1
rc=$?; tail -2 $O/r4c3_tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/r4c3_tests.log | head -20; exit $rc; }
for i in 1 2; do
  for L in 0 1; do
    MPA_BN_LINK=$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 --small-batch 0 > $O/r4c3_link$L.$i.json 2> $O/r4c3_link$L.$i.err || { echo "bench L=$L failed"; tail -5 $O/r4c3_link$L.$i.err; exit 1; }
    python -c "import json; d=json.load(open('$O/r4c3_link$L.$i.json')); print('link=$L', d['value'], d['ms_per_step'])"
  done
done
cd /tmp
B="python3 $R/bench.py --steps 2 --warmup 1 --small-batch 0"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-trace --output-format csv -d $R/$O/c3pmc1 -o p -- $B > $R/$O/c3pmc1.log 2>&1 || { echo pmc1 failed; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA TA_BUSY_avr TCC_HIT_sum --kernel-trace --output-format csv -d $R/$O/c3pmc2 -o p -- $B > $R/$O/c3pmc2.log 2>&1 || { echo pmc2 failed; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/$O/c3pmc3 -o p -- $B > $R/$O/c3pmc3.log 2>&1 || { echo pmc3 failed; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/$O/c3pmc4 -o p -- $B > $R/$O/c3pmc4.log 2>&1 || { echo pmc4 failed; exit 1; }
cd $R
python3 tools/pmc_summary.py $(find $O/c3pmc1 $O/c3pmc2 $O/c3pmc3 $O/c3pmc4 -name "*counter_collection.csv") > $O/r4c3_pmc_summary.txt
find $O/c3pmc1 $O/c3pmc2 $O/c3pmc3 $O/c3pmc4 -name "*.csv" -size +2M -delete
grep -A3 "conv3_halo_kernel<true, 8" $O/r4c3_pmc_summary.txt | head -8
timeout -k 10 600 python -u -m pytest tests/test_eval_pipeline_gpu.py -x -q -k zoo --timeout 300 --timeout-method thread -p no:cacheprovider > $O/r4c3_evaltests.log 2>&1
rc=$?; tail -2 $O/r4c3_evaltests.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/r4c3_evaltests.log | head -20; exit $rc; }
for cfg in "resnet18 224 224" "resnet18 224 448" "inception 299 299" "densenet 224 224"; do
  set -- $cfg
  MODEL=$1 HW=$2 timeout -k 10 300 python tools/bench_eval.py 20480 256 1,2,3 $3 >> $O/r4c3_eval.txt 2>> $O/r4c3_eval.err || { echo "eval $cfg failed"; tail -3 $O/r4c3_eval.err; exit 1; }
done
cat $O/r4c3_eval.txt
timeout -k 10 600 python -u -m pytest tests/test_models_gpu.py tests/test_layer_parity_gpu.py -x -q -k "vgg or alexnet" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/r4c3_vggtests.log 2>&1
rc=$?; tail -2 $O/r4c3_vggtests.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/r4c3_vggtests.log | head -20; exit $rc; }
for L in 1 0; do
  MPA_SEQ_LINK=$L timeout -k 10 300 python bench.py --model vgg16 --batch 256 --steps 10 --warmup 3 --small-batch 0 > $O/r4c3_vgg_$L.json 2> $O/r4c3_vgg_$L.err || { tail -3 $O/r4c3_vgg_$L.err; exit 1; }
  python -c "import json; print('vgg16 seqlink=$L', json.load(open('$O/r4c3_vgg_$L.json'))['value'])"
done
timeout -k 10 900 python -u -m pytest tests/test_models_gpu.py tests/test_grouped_gpu.py tests/test_layer_parity_gpu.py tests/test_kernels_gpu.py -x -q -k "inception or densenet or grouped or bn" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/r4c3_inctests.log 2>&1
rc=$?; tail -2 $O/r4c3_inctests.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/r4c3_inctests.log | head -20; exit $rc; }
for L in 1 0; do
  MPA_CAT_INTO=$L timeout -k 10 300 python bench.py --model inception --image-size 299 --batch 256 --steps 10 --warmup 3 --small-batch 0 > $O/r4c3_inc_$L.json 2> $O/r4c3_inc_$L.err || { tail -3 $O/r4c3_inc_$L.err; exit 1; }
  python -c "import json; print('inception catinto=$L', json.load(open('$O/r4c3_inc_$L.json'))['value'])"
done
timeout -k 10 300 python bench.py --model densenet --batch 256 --steps 10 --warmup 3 --small-batch 0 > $O/r4c3_dense.json 2> $O/r4c3_dense.err || { tail -3 $O/r4c3_dense.err; exit 1; }
python -c "import json; print('densenet', json.load(open('$O/r4c3_dense.json'))['value'])"
