"""Same-box A/B of the measured GEMM shape table (tao_tune_gemm_table 0 / 1) on the shapes the
e2e prefill and bench.py run: kernel us, table on vs off, alternated twice.

    python experiments/ab_table.py
"""
import json

from sweep_gemm import kernel_us, make_int4, make_int8dyn, make_int8wo
from torchao import _lib

CONFIGS = [("int4", 128, 4096, 4096), ("int4", 128, 6144, 4096), ("int4", 128, 28672, 4096),
           ("int4", 128, 4096, 14336), ("int4", 64, 6144, 4096), ("int4", 512, 28672, 4096),
           ("int8dyn", 128, 4096, 4096), ("int8dyn", 64, 6144, 4096),
           ("int8wo", 128, 28672, 4096), ("int8wo", 128, 128256, 4096)]


def main():
    mk = {"int4": make_int4, "int8wo": make_int8wo, "int8dyn": make_int8dyn}
    _lib.call("tao_tune_linear_crossover", 1)
    for path, M, N, K in CONFIGS:
        run, launches = mk[path](M, N, K)
        res = {"on": [], "off": []}
        for _ in range(2):
            for key, off in (("on", 0), ("off", 1)):
                _lib.call("tao_tune_gemm_table", off)
                res[key].append(round(kernel_us(run, launches, reps=30), 2))
        _lib.call("tao_tune_gemm_table", 0)
        print(json.dumps({"path": path, "M": M, "N": N, "K": K, "table_us": res["on"],
                          "heuristic_us": res["off"]}), flush=True)


if __name__ == "__main__":
    main()
