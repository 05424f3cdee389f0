export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 900 bash experiments/tile_debug.sh run > $O/tile_debug6.txt 2>&1
