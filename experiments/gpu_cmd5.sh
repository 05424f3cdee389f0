export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 1000 python -u experiments/ab_tile.py > $O/ab_tile_full.jsonl 2> $O/ab_tile_full.err
