"""A/B the decode-attention kernels end to end: for each tao_tune_attn mode, alternating, run the
e2e harness (torchao._models.llama.generate) and print its JSON line.
Usage: python experiments/ab_attn.py [-q int4wo-32] [--modes 0,1] [--rounds 2]"""

import argparse
import io
import json
import os
import sys
from contextlib import redirect_stdout

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "torchao-fork_amd"))

from torchao import _lib  # noqa: E402
from torchao._models.llama import generate  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-q", default="int4wo-32")
    ap.add_argument("--modes", default="0,2,3")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--max_new_tokens", type=int, default=200)
    a = ap.parse_args()
    for r in range(a.rounds):
        for mode in [int(m) for m in a.modes.split(",")]:
            _lib.call("tao_tune_attn", mode)
            buf = io.StringIO()
            with redirect_stdout(buf):
                generate.main(["-q", a.q, "--num_samples", "3",
                               "--max_new_tokens", str(a.max_new_tokens)])
            rec = json.loads(buf.getvalue().strip().splitlines()[-1])
            print(json.dumps({"attn_mode": mode, "round": r,
                              "decode_tokens_per_s": rec.get("decode_tokens_per_s"),
                              "decode_ms_per_token": rec.get("decode_ms_per_token")}), flush=True)


if __name__ == "__main__":
    main()
