"""Print VGPRs / scratch / occupancy per kernel of the HIP sources (hipcc remarks)."""
import re, subprocess, sys
srcs = sys.argv[1:] or ["int4_gemv.hip", "int8_gemv.hip", "gemm_mfma.hip", "int8_dyn.hip", "int4_pack.hip"]
for s in srcs:
    out = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950",
                          "-Rpass-analysis=kernel-resource-usage", "-c", s, "-o", "/dev/null"],
                         capture_output=True, text=True).stderr
    cur = {}
    for line in out.splitlines():
        m = re.search(r"remark:\s+(Function Name|VGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]): (\S+)", line)
        if not m:
            continue
        k, v = m.group(1).split()[0], m.group(2)
        if k == "Function":
            name = re.sub(r"^_ZN3tao12_GLOBAL__N_1\d+", "", v)
            cur = {"name": re.sub(r"E+vPK.*|Ev.*$", "", name)}
        else:
            cur[k] = v
        if k == "Occupancy":
            print(f"{cur['name'][:60]:60s} vgpr={cur.get('VGPRs')} scratch={cur.get('ScratchSize')} occ={v}")
