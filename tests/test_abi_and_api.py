"""CPU-side checks: the C-ABI library loads and exports every symbol include/csu.h declares, the
ctypes struct layouts match the header, the nn.Module surface matches the reference's
state_dict contract (fixture F7), and the product path refuses CPU tensors (no fallback)."""
import ctypes
import json
import os
import re

import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(REPO, "include", "csu.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(csu_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    from csu import _lib
    L = _lib.lib()
    names = header_functions()
    assert len(names) >= 10
    for n in names:
        assert hasattr(L, n), n
        assert n in _lib._SIGS, f"{n} missing from the ctypes signature table"
    assert b"gfx950" in L.csu_build_info()


def test_gemm_ws_rejects_unwritable_out_dtype():
    """the weight-streaming GEMM's support query sees the real output dtype (fp16 or any
    non-fp32 / bf16 dtype is rejected, so the caller falls back instead of failing in gemm_ws)."""
    from csu import ops
    assert ops.dtype_code_of(torch.float16) == -1 and ops.dtype_code_of(torch.bfloat16) == 1
    assert ops._ws_ok(1024, 768, 256, torch.bfloat16) and ops._ws_ok(1024, 768, 256, torch.float32)
    assert not ops._ws_ok(1024, 768, 256, torch.float16)


def test_struct_layout_matches_header(tmp_path):
    """The ctypes mirrors of the C structs have the C compiler's sizes and field offsets
    (include/csu.h compiled by gcc here)."""
    import subprocess
    from csu import _lib
    checks = {"csu_stripe_branch": (_lib.StripeBranch, ["H_sp", "ch_off", "lepe_w", "lepe_db"]),
              "csu_stripe_args": (_lib.StripeArgs, ["scale", "br", "drop_rng", "drop_site", "drop_p"]),
              "csu_gemm_desc": (_lib.GemmDesc, ["M", "a", "b_trans", "bias", "out", "ldc", "cfg"]),
              "csu_mlp_dropout": (_lib.MlpDropout, ["rng", "site_out", "p", "row_scale", "rows_per_sample"]),
              "csu_conv_geom": (_lib.ConvGeom, ["B", "KH", "pad"]),
              "csu_wslab_item": (_lib.WslabItem, ["slab", "dst", "N", "tk", "chunks"]),
              "csu_wgrad_group_item": (_lib.WgradGroupItem, ["dy", "x", "dw_db", "slab", "M", "N", "K"]),
              "csu_ln_param_item": (_lib.LnParamItem, ["workspace", "dbeta", "rows", "C"])}
    lines = ["#include <stdio.h>", "#include <stddef.h>", '#include "csu.h"', "int main(void) {"]
    for cname, (_, fields) in checks.items():
        lines.append(f'printf("{cname} %zu\\n", sizeof({cname}));')
        for f in fields:
            lines.append(f'printf("{cname}.{f} %zu\\n", offsetof({cname}, {f}));')
    lines.append("return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    inc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include")
    subprocess.run(["gcc", "-I", inc, str(src), "-o", str(exe)], check=True)
    got = dict(line.split() for line in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.splitlines())
    for cname, (cls, fields) in checks.items():
        assert ctypes.sizeof(cls) == int(got[cname]), cname
        for f in fields:
            assert getattr(cls, f).offset == int(got[f"{cname}.{f}"]), (cname, f)


def test_error_path_reports_text():
    from csu import _lib
    L = _lib.lib()
    a = _lib.StripeArgs()
    a.head_dim = 16   # unsupported -> CSU_E_UNSUPPORTED before any device work
    rc = L.csu_stripe_attn_fwd(ctypes.byref(a), 0, None, None, None, None)
    assert rc == -2
    assert b"head_dim" in L.csu_last_error_string()
    rc = L.csu_layernorm_fwd(4, 96, 1e-5, 0, None, None, None, 0, None, None, None, None)
    assert rc == -2


@pytest.mark.parametrize("name,kw", [("default_224", dict(img_size=224)),
                                     ("cfg512", dict(img_size=512, split_size=[1, 2, 8, 8])),
                                     ("deep512", dict(img_size=512, depth=[2, 4, 32, 2], split_size=[1, 2, 8, 8]))])
def test_state_dict_contract_matches_reference(golden_dir, name, kw):
    from csu.model import CSWinTransformer
    ref = json.load(open(os.path.join(golden_dir, "f7_contract.json")))[name]
    m = CSWinTransformer(**kw)
    assert [[k, list(v.shape)] for k, v in m.state_dict().items()] == ref
    m2 = CSWinTransformer(simam=True, **kw)
    assert list(m2.state_dict().keys()) == [k for k, _ in ref]


def test_reference_init_statistics():
    """_init_weights (cswin:607-614): Linear ~ trunc N(0, .02), zero bias; LN (1, 0)."""
    from csu.model import CSWinTransformer
    torch.manual_seed(0)
    m = CSWinTransformer(img_size=128, split_size=[1, 2, 4, 4])
    w = m.stage3[0].mlp.fc1.weight
    assert abs(float(w.std()) - 0.02) < 2e-3 and float(m.stage3[0].mlp.fc1.bias.abs().max()) == 0
    assert float((m.norm.weight - 1).abs().max()) == 0


def test_product_refuses_cpu_tensors():
    from csu import ops
    from csu._lib import CsuError
    geom = ops.StripeGeometry(8, 32, 1, [(8, 1, 0)], 32 ** -0.5)
    with pytest.raises(CsuError):
        ops.stripe_attention(torch.zeros(1, 64, 96), geom, [torch.zeros(32, 1, 3, 3)], [torch.zeros(32)])
    with pytest.raises(CsuError):
        ops.layer_norm(torch.zeros(4, 64), torch.ones(64), torch.zeros(64))


def test_geometry_validation_mirrors_reference():
    from csu import ops
    with pytest.raises(ValueError):   # img2windows view fails when reso % split != 0 (cswin:204)
        ops.StripeGeometry(16, 64, 2, [(16, 7, 0)], 0.1)


@pytest.mark.parametrize("img,depth", [(512, [1, 2, 9, 1]), (512, [2, 4, 32, 2]), (1024, [1, 2, 9, 1]), (256, [1, 2, 9, 1])])
def test_default_split_rejected_where_reference_crashes(img, depth):
    """The reference default split_size [1,2,7,7] (cswin:494) cannot run at 256/512/1024: the
    stage-3 resolution img/16 is not a multiple of 7 and img2windows' view fails (cswin:204, SURVEY
    0.4) -- including BASELINE config 4 (deep, 512).  csu rejects the model at construction with the
    same cause; [1,2,8,8] builds (no device work happens in __init__)."""
    from csu.model import CSWinTransformer
    with pytest.raises(ValueError, match="not divisible"):
        CSWinTransformer(img_size=img, depth=depth, split_size=[1, 2, 7, 7])
    CSWinTransformer(img_size=img, depth=depth, split_size=[1, 2, 8, 8])


def test_dice_iou_metrics_match_reference_fixture(golden_dir):
    import numpy as np
    from csu.train import bce_loss, dice_coefficient, iou_score
    z = np.load(os.path.join(golden_dir, "f5_metrics.npz"))
    p, t = torch.from_numpy(z["p"]), torch.from_numpy(z["t"])
    pred = (p > 0.5).float()
    assert abs(dice_coefficient(pred, t) - float(z["dice"])) < 1e-7
    assert abs(iou_score(pred, t) - float(z["iou"])) < 1e-7
    assert abs(bce_loss(p, t).item() - float(z["bce"])) < 1e-6
