"""Where does the fused Mlp at C = 256 (16384 tokens: stage 3 at 512x512 B16) spend its time?
Ablation builds of csrc/mlp.hip (text edits on a copy; the product source is untouched), each linked
with common.o into a small library, and the forward / backward timed on the GPU:

    python tools/probes/mlp_ablate.py build     # here (hipcc): tools/probes/mlp_abl/<variant>.so
    python tools/probes/mlp_ablate.py run       # on the GPU box: one line per variant

Variants (each removes one component of the per-chunk chain; results are wrong by design):
  base     the product kernels
  nodma    no weight DMA inside the chunk loop (the prologue's chunks are re-read: LDS-resident weights)
  nosync   nodma + no vmcnt wait / barrier per chunk (the compute chain alone)
  nogelu   GELU (forward) / GELU + GELU' (backward) replaced by an add
  nomfma   the MFMAs removed (fragment reads kept live)
  nostore  (backward) no g / dH global stores"""
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
CSRC = os.path.join(REPO, "cswin-simam-unet_amd", "csrc")
OUT = os.path.join(HERE, "mlp_abl")
# round 6 set: "old" = the 4-wave kernels (the ablations of those, base / nodma / nosync / nogelu / nomfma /
# nostore, are in profiles/r08b_mlp_ablate.txt), "w8" = the 8-wave kernels as built, and their ablations
VARIANTS = ["old", "w8", "w8_hc64", "w8_nodma", "w8_nomfma", "w8_dmaonly"]
# per-phase ablations of the 8-wave backward (phase A / B / C of mlp_bwd8_kernel skipped, one at a time)
if os.environ.get("MLP_ABL_SET") == "bwd8":
    VARIANTS = ["w8", "w8_nodma", "w8_noA", "w8_noB", "w8_noC", "w8_noAC", "w8_dmaonly"]
OLD_ONLY = ("base", "nodma", "nosync", "nogelu", "nomfma", "nostore", "old")


def edit(src: str, v: str) -> str:
    if v == "w8":
        return src
    if v in OLD_ONLY:   # C = 256 dispatches to the 4-wave kernels
        assert src.count("if (!d) {   // two waves per SIMD") == 2
        src = src.replace("if (!d) {   // two waves per SIMD", "if (false) {   // two waves per SIMD")
    if v.startswith("w8_"):   # the 8-wave C = 256 kernels (mlp_fwd8_kernel / mlp_bwd8_kernel)
        a = src.index("// Forward at C = 256 with two waves per SIMD")
        b = src.index("template <int C>\nint fwd_launch(")
        body = src[a:b]
        if v == "w8_hc64":        # (name kept from r08f) the other chunk size: 32-hidden chunks, 4-stage ring
            return src.replace("constexpr int kFwd8Hc = 64;", "constexpr int kFwd8Hc = 32;")
        if v == "w8_nodma":
            body = body.replace("if (j + NST - 1 < NCH) dma1(", "if (false) dma1(").replace("if (j + NST - 2 < NCH) dma2(", "if (false) dma2(")
            body = body.replace("if (j + 1 < NCH) {\n            dma", "if (false) {\n            dma")
        if v in ("w8_nomfma", "w8_dmaonly"):
            body = re.sub(r"(\w+(?:\[\w+\])*) = __builtin_amdgcn_mfma_f32_(?:32x32x16|16x16x32)_bf16\(([^;]*?), ([\w\[\]]+), \1, 0, 0, 0\);",
                          r'asm volatile("" :: "v"(\2), "v"(\3));', body)
        phases = {"A": "// ---- phase A\n        {", "B": "// ---- phase B\n        {",
                  "C": "// ---- phase C: acc[tt] += W1[chunk]^T[fo ..][hidden] dH[hidden][32 tt ..]\n        {"}
        if v in ("w8_noA", "w8_noB", "w8_noC", "w8_noAC"):
            for k in v[len("w8_no"):]:
                assert phases[k] in body, k
                body = body.replace(phases[k], phases[k].replace("{", "if (M < 0) {"))
            return src[:a] + body + src[b:]
        if v == "w8_dmaonly":     # DMA + barriers only: no fragment reads, no GELU, no phase work
            body = body.replace("if (j < NCH) gemm1(j);", "").replace("if (j > 0) gemm2(j - 1);", "")
            for ph in ("// ---- phase A\n        {", "// ---- phase B\n        {", "// ---- phase C: acc[tt] += W1[chunk]^T[fo ..][hidden] dH[hidden][32 tt ..]\n        {"):
                assert ph in body, ph
                body = body.replace(ph, ph.replace("{", "if (M < 0) {"))
        return src[:a] + body + src[b:]
    a = src.index("__global__ __launch_bounds__(MT) void mlp_fwd_kernel")
    b = src.index("// Persistent backward for C = 64")
    body = src[a:b]
    if v in ("nodma", "nosync"):
        body = body.replace("if (j + 2 < NCH) dma<D1::NW>", "if (false) dma<D1::NW>")
        body = body.replace("if (j + 1 < NCH) dma<D2::NW>", "if (false) dma<D2::NW>")
        body = body.replace("if (j + 2 < NCH) {\n                dma", "if (false) {\n                dma")
        body = body.replace("if (j + 1 < NCH) {\n                dma", "if (false) {\n                dma")
    if v == "nosync":
        body = re.sub(r"vmwait<0>\(\);\s+// W1\(j\+1\).*", "", body)
        body = re.sub(r"lds_sync\(\);\s+// every wave is past GEMM1\(j\).*", "", body)
        body = body.replace("if (j == 0) vmwait<0>(); else vmwait<8>();", "if (j == 0) vmwait<0>();")
        body = re.sub(r"lds_sync\(\);\s+// every wave is past chunk j-1.*", "if (j == 0) lds_sync();", body)
    if v == "nogelu":
        body = body.replace("gv[e] = gelu_fast(cur[e] + bv[e]);", "gv[e] = cur[e] + bv[e];")
        body = body.replace("gelu_pair_fast(hc[e] + bv[e], gv[e], dg);", "gv[e] = hc[e] + bv[e]; dg = hc[e];")
    if v == "nomfma":
        body = re.sub(r"(\w+(?:\[\w+\])?) = __builtin_amdgcn_mfma_f32_32x32x16_bf16\(([^;]*?), (\w+(?:\[[\w +]+\])?), \1, 0, 0, 0\);",
                      r'asm volatile("" :: "v"(\2), "v"(\3));', body)
    if v == "nostore":
        body = body.replace("buf_st4bf(rs_g, o, gv + 4 * g);", "")
        body = body.replace("buf_st4bf(rs_dh, o, dv + 4 * g);", "")
    return src[:a] + body + src[b:]


def build():
    os.makedirs(OUT, exist_ok=True)
    src = open(os.path.join(CSRC, "mlp.hip")).read()
    flags = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", f"-I{os.path.join(REPO, 'include')}", f"-I{CSRC}",
             "-mllvm", "-amdgpu-mfma-vgpr-form"]
    common = os.path.join(OUT, "common.o")
    subprocess.run(["hipcc", *flags, "-x", "hip", "-c", os.path.join(CSRC, "common.cpp"), "-o", common], check=True)
    for v in VARIANTS:
        s = edit(src, v)
        if v != "w8":
            assert s != src, v
        p = os.path.join(OUT, f"mlp_{v}.hip")
        open(p, "w").write(s)
        o = p.replace(".hip", ".o")
        subprocess.run(["hipcc", *flags, "-c", p, "-o", o], check=True)
        subprocess.run(["hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", o, common, "-o",
                        os.path.join(OUT, f"{v}.so")], check=True)
        os.remove(p)
        os.remove(o)
        print("built", v, flush=True)
    os.remove(common)


def run():
    import ctypes
    import torch
    d = torch.device("cuda:0")
    C, M = 256, 16384
    g = torch.Generator(device=d).manual_seed(0)
    x = torch.randn(M, C, device=d, generator=g).bfloat16()
    w1 = (torch.randn(4 * C, C, device=d, generator=g) * C ** -0.5).bfloat16()
    w2 = (torch.randn(C, 4 * C, device=d, generator=g) * (4 * C) ** -0.5).bfloat16()
    b1, b2 = torch.zeros(4 * C, device=d), torch.zeros(C, device=d)
    res, y = torch.randn(M, C, device=d, generator=g), torch.empty(M, C, device=d)
    dy = torch.randn(M, C, device=d, generator=g).bfloat16()
    dh = torch.empty(M, 4 * C, device=d, dtype=torch.bfloat16)
    gg = torch.empty(M, 4 * C, device=d, dtype=torch.bfloat16)
    dx = torch.empty(M, C, device=d, dtype=torch.bfloat16)
    P = lambda t: ctypes.c_void_p(t.data_ptr())   # noqa: E731
    st = ctypes.c_void_p(torch.cuda.current_stream(d).cuda_stream)

    def timeit(fn, n=50):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(n):
            fn()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / n * 1e3

    for v in VARIANTS:
        L = ctypes.CDLL(os.path.join(OUT, f"{v}.so"))
        L.csu_mlp_fwd.restype = L.csu_mlp_bwd.restype = ctypes.c_int
        L.csu_mlp_fwd.argtypes = [ctypes.c_long, ctypes.c_int] + [ctypes.c_void_p] * 7 + [ctypes.c_void_p]
        L.csu_mlp_bwd.argtypes = [ctypes.c_long, ctypes.c_int] + [ctypes.c_void_p] * 8 + [ctypes.c_void_p]
        f = timeit(lambda: L.csu_mlp_fwd(M, C, P(x), P(w1), P(b1), P(w2), P(b2), P(res), P(y), st))
        bw = timeit(lambda: L.csu_mlp_bwd(M, C, P(x), P(dy), P(w1), P(b1), P(w2), P(dh), P(gg), P(dx), st))
        one = timeit(lambda: L.csu_mlp_fwd(64, C, P(x), P(w1), P(b1), P(w2), P(b2), P(res), P(y), st))
        oneb = timeit(lambda: L.csu_mlp_bwd(64, C, P(x), P(dy), P(w1), P(b1), P(w2), P(dh), P(gg), P(dx), st))
        print(f"{v:8s} fwd {f:6.1f} us (one workgroup {one:5.1f})   bwd {bw:6.1f} us (one workgroup {oneb:5.1f})", flush=True)


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
