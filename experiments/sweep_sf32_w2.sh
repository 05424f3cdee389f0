export PYTHONPATH=torchao-fork_amd TMPDIR=/tmp
O=gpurun_out/r5k_sf32_w2.jsonl
: > $O
for spec in "128x4096x14336 64,2,4,4,0,0 0" "128x4096x14336 128,1,8,3,0,1 2" "128x4096x14336 128,1,4,3,0,2 2" "128x4096x14336 128,1,8,3,0,2 2" "128x4096x14336 64,1,8,3,0,1 2" "128x4096x14336 64,1,16,3,0,1 2" "128x4096x4096 64,2,4,4,0,0 0" "128x4096x4096 128,1,4,3,0,1 2" "128x4096x4096 128,1,8,3,0,1 2" "128x4096x4096 64,1,4,3,0,1 2" "128x4096x4096 128,1,4,3,0,2 2"; do
  set -- $spec
  timeout -k 10 120 python -u experiments/time_sf_cfg.py int4 $1 $2 $3 >> $O 2>> gpurun_out/r5k_sf32_w2.err || exit $?
done
cat $O
