set -e
bash scripts/gpu/run.sh a3 tests=pre_bn
MPA_BN_PRE=1 bash scripts/gpu/run.sh a3p1 "seq=--wgrad-stream,0"
MPA_BN_PRE=0 bash scripts/gpu/run.sh a3p0 "seq=--wgrad-stream,0"
MPA_BN_PRE=0 MPA_HALO_WPROD=1 bash scripts/gpu/run.sh a3wp "seq=--wgrad-stream,0"
bash scripts/gpu/run.sh a3 "ab=MPA_BN_PRE=0|--wgrad-stream 0;MPA_BN_PRE=1|--wgrad-stream 0;MPA_BN_PRE=0 MPA_HALO_WPROD=1|--wgrad-stream 0;MPA_BN_PRE=0;MPA_BN_PRE=1"
bash scripts/gpu/run.sh a3g "gaps=--batch,128" "gaps=--batch,128,--graph,on" "gaps=--batch,128,--wgrad-stream,0"
