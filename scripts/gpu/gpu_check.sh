#!/bin/bash
# GPU session runner: scripts/gpu/gpu_check.sh step1 step2 ...  Steps: kernels models smoke bench prof diag
# Stops at the first crash/timeout (pytest rc 1 = test failures only, continue).
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1; local t=$2; shift 2; timeout -k 10 "$t" "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -4 gpurun_out/$name.log; return $rc; }
for step in "$@"; do
  case $step in
    kernels) run kernels 900 python -m pytest tests/test_kernels_gpu.py -q -p no:cacheprovider; rc=$? ;;
    models) run models 900 python -m pytest tests/test_models_gpu.py -q -p no:cacheprovider; rc=$? ;;
    gputests) run gputests 1200 python -m pytest tests -m gpu -q -p no:cacheprovider; rc=$? ;;
    smoke) run smoke 300 python __graft_entry__.py smoke; rc=$? ;;
    bench) run bench 600 python bench.py --steps 20 --warmup 5; rc=$? ;;
    losses) run losses_g 300 python bench.py --steps 30 --warmup 2 --print-losses && MPA_NO_STATS_SHIFT=1 run losses_ns 300 python bench.py --steps 30 --warmup 2 --print-losses && run losses_e 300 python bench.py --steps 30 --warmup 2 --print-losses --graph off; rc=$? ;;
    benchab) run benchab_g 300 python bench.py --steps 10 --warmup 3 --graph on && run benchab_e 300 python bench.py --steps 10 --warmup 3 --graph off && MPA_NO_STATS_SHIFT=1 run benchab_ns 300 python bench.py --steps 10 --warmup 3 --graph on; rc=$? ;;
    bench128) run bench128 600 python bench.py --steps 20 --warmup 5 --batch 128; rc=$? ;;
    benchnog) run benchnog 600 python bench.py --steps 20 --warmup 5 --graph off; rc=$? ;;
    prof) run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o r18 --output-format csv -- python bench.py --steps 5 --warmup 2 --graph off; rc=$? ;;
    benchk) run benchk 600 python tools/bench_kernels.py 256 10; rc=$? ;;
    benchk1) MPA_BENCH_ENGINES=1 run benchk1 600 python tools/bench_kernels.py 256 10; rc=$? ;;
    sweep) run sweep 900 python tools/bench_kernels.py 256 5 sweep; rc=$? ;;
    dp2) MPA_DIST_BACKEND=gloo run dp2 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 2 --steps 5 --warmup 2 --batch 64; rc=$? ;;
    dp2t) MPA_DIST_BACKEND=gloo run dp2t 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29556 tools/dp_check.py; rc=$? ;;
    zoo) for m in "resnet34 224 256" "vgg16 224 128" "inception 299 128" "densenet 224 128" "alexnet 224 256" "squeezenet 224 256" "vgg 224 128"; do set -- $m; timeout -k 10 300 python bench.py --model $1 --image-size $2 --batch $3 --steps 10 --warmup 3 >> gpurun_out/zoo.log 2>&1 || { echo "zoo $1 failed rc=$?"; exit 1; }; done; rc=0 ;;
    profinc) run profinc 600 rocprofv3 --kernel-trace --stats -d gpurun_out/profinc -o inc --output-format csv -- python bench.py --model inception --image-size 299 --batch 128 --steps 3 --warmup 2; rc=$? ;;
    zoo2) for m in "squeezenet 224 256" "inception 299 128"; do set -- $m; timeout -k 10 300 python bench.py --model $1 --image-size $2 --batch $3 --steps 10 --warmup 3 >> gpurun_out/zoo2.log 2>&1 || { echo "zoo $1 failed rc=$?"; exit 1; }; done; rc=0 ;;
    linkab) MPA_BN_LINK=0 run link0 300 python bench.py --steps 20 --warmup 5 && MPA_BN_LINK=1 run link1 300 python bench.py --steps 20 --warmup 5 && MPA_BN_LINK=0 run link0b 300 python bench.py --steps 20 --warmup 5 && MPA_BN_LINK=1 run link1b 300 python bench.py --steps 20 --warmup 5; rc=$? ;;
    stemab) MPA_NO_STEM_FUSE=1 run stem0 300 python bench.py --steps 20 --warmup 5 && run stem1 300 python bench.py --steps 20 --warmup 5 && MPA_NO_STEM_FUSE=1 run stem0b 300 python bench.py --steps 20 --warmup 5 && run stem1b 300 python bench.py --steps 20 --warmup 5; rc=$? ;;
    stemgrid) for f in 1024 4096; do for r in 512 1024 2048; do for a in 1024 4096; do echo "F=$f R=$r A=$a" >> gpurun_out/stemgrid.log; MPA_STEM_GRID_F=$f MPA_STEM_GRID_R=$r MPA_STEM_GRID_A=$a timeout -k 10 120 python bench.py --steps 20 --warmup 5 >> gpurun_out/stemgrid.log 2>&1 || exit 1; done; done; done; rc=0 ;;
    diag) run diag 600 python tools/diag_grads.py; rc=$? ;;
    benchbn) for g in 0 256 512 1024; do for u in 1; do MPA_BN_GRID=$g MPA_BN_UNR=$u timeout -k 10 120 python tools/bench_bn.py 20 >> gpurun_out/benchbn.log 2>&1 || exit 1; done; done; rc=0 ;;
    diageng) run diageng 600 python tools/diag_engines.py inception 299 4; rc=$? ;;
    diag2) run diag2 600 python tools/diag_grads.py twice; rc=$? ;;
    traj) run traj 600 python tools/diag_traj.py 64 25 && MPA_NO_STATS_SHIFT=1 timeout -k 10 600 python tools/diag_traj.py 64 25 > gpurun_out/traj_noshift.log 2>&1; rc=$? ;;
    train) run train 600 python main.py --synthetic_images 2048 --image_size 224 --NUM_EPOCHS 2 --BATCH_SIZE 256 --CHECKPOINT_DIR /tmp/mpa_ck/ --log_file gpurun_out/training.log; rc=$? ;;
    evalp) run evalp 600 python evaluation_pipeline.py --synthetic_images 16384 --image_size 224 --eval_lanes 3 --eval_batch 256 --CHECKPOINT_DIR /tmp/mpa_ck/ --log_file gpurun_out/evaluation.log; rc=$? ;;
    *) echo "unknown step $step"; rc=0 ;;
  esac
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $step rc=$rc"; exit $rc; fi
done
