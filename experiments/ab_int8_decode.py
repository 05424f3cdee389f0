"""e2e int8wo decode under launch-shape overrides of the int8 GEMVs (tao_tune_int8_gemv: rows per
wave, waves along K, row groups; applies to the fused decode kernel and the plain int8 GEMV).
python experiments/ab_int8_decode.py"""
import io
import json
import os
import sys
from contextlib import redirect_stdout

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "torchao-fork_amd"))
from torchao import _lib  # noqa: E402
from torchao._models.llama import generate  # noqa: E402

CONFIGS = [(0, 0, 0), (4, 4, 1), (8, 4, 2), (2, 4, 2), (0, 0, 0)]
for rpw, wk, g in CONFIGS:
    _lib.call("tao_tune_int8_gemv", rpw, wk, g)
    buf = io.StringIO()
    with redirect_stdout(buf):
        generate.main(["-q", "int8wo", "--num_samples", "2"])
    line = [l for l in buf.getvalue().splitlines() if l.startswith("{")][-1]
    d = json.loads(line)
    print(json.dumps({"tune": [rpw, wk, g], "decode_tokens_per_s": d["decode_tokens_per_s"]}),
          flush=True)
_lib.call("tao_tune_reset")
