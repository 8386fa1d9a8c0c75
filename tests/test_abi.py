"""CPU tests of the C-ABI boundary: libtic.so loads, exports exactly what include/tic.h
declares, its layer tables agree with the host mirror and with the oracle's independent
tables, and argument validation fails loudly without touching a device."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from conftest import ROOT
from oracle import tic_oracle as o

HEADER = os.path.join(ROOT, "include", "tic.h")


def header_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(tic_[a-z0-9_]+)\s*\(", txt)))


@pytest.fixture(scope="module")
def L():
    from tf_image_compression_amd import _lib
    return _lib.lib()


def test_library_exports_every_header_symbol(L):
    names = header_functions()
    assert len(names) >= 25
    for n in names:
        assert hasattr(L, n), f"{n} declared in include/tic.h but not exported"


def test_binding_covers_header():
    from tf_image_compression_amd import _lib
    bound = {n for n, _, _ in _lib.SIGNATURES}
    assert bound == set(header_functions())


def test_exports_are_c_symbols():
    import subprocess
    out = subprocess.run(["nm", "-D", "--defined-only", os.path.join(ROOT, "tf_image_compression_amd", "libtic.so")],
                         capture_output=True, text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    for n in header_functions():
        assert n in exported  # unmangled: extern "C"


def _native_table(L, model_id):
    out = []
    for i in range(L.tic_model_num_layers(model_id)):
        name = C.create_string_buffer(128)
        v = [C.c_int() for _ in range(6)]
        assert L.tic_model_layer(model_id, i, name, 128, *[C.byref(x) for x in v]) == 0
        out.append((name.value.decode(), *[x.value for x in v]))
    return out


@pytest.mark.parametrize("model_id", [0, 1, 2, 3, 128, 100])
def test_native_table_matches_host_and_oracle(L, model_id):
    from tf_image_compression_amd.topology import layer_table
    kinds = {"conv_s1": 0, "conv_s2": 1, "convT": 2}
    host = [(l.name, kinds[l.kind], l.cin, l.cout, 1 if l.act == "relu" else 0, 0 if l.stage == "enc" else 1,
             int(l.residual)) for l in layer_table(model_id)]
    assert _native_table(L, model_id) == host
    # the oracle's independently written tables: same TF variable names and shapes
    if model_id == 100:
        shapes = o.param_shapes(o.RMBE)
    else:
        shapes = o.param_shapes(o.MODELS[model_id][0] + o.MODELS[model_id][1])
    from tf_image_compression_amd.topology import param_shapes
    assert param_shapes(model_id) == shapes


def test_argument_errors_without_device(L):
    h = C.c_void_p()
    assert L.tic_create(7, 256, 2, 0, C.byref(h)) == -1
    assert b"unknown model" in L.tic_last_error()
    assert L.tic_create(0, 255, 2, 0, C.byref(h)) == -1
    assert L.tic_create(0, 256, 1, 0, C.byref(h)) == -1
    assert L.tic_create(0, 256, 300, 0, C.byref(h)) == -1
    assert L.tic_create(0, 200, 2, 0, C.byref(h)) == -1
    assert b"divisible" in L.tic_last_error()
    assert L.tic_model_num_layers(99) == -1
    assert L.tic_encode(None, None, 1, None, None) == -1
    assert L.tic_decode(None, None, 1, None, None) == -1
    assert L.tic_set_param(None, b"x", None, None, 0) == -1
    assert L.tic_finalize(None) == -1
    assert L.tic_synchronize(None) == -1


def test_python_wrapper_raises_not_falls_back(monkeypatch):
    """No CPU fallback: a missing library is a hard error."""
    from tf_image_compression_amd import _lib
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", "/nonexistent/libtic.so")
    with pytest.raises(_lib.TicError):
        _lib.lib()


def test_product_package_never_imports_oracle():
    """The oracle is test infrastructure: no product module may reference it."""
    pkg = os.path.join(ROOT, "tf_image_compression_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(".py"):
                src = open(os.path.join(dirpath, f)).read()
                assert not re.search(r"^\s*(from|import)\s+oracle", src, re.M), f
    for f in ("encode.py", "decode.py"):
        p = os.path.join(ROOT, f)
        if os.path.exists(p):
            assert not re.search(r"^\s*(from|import)\s+oracle", open(p).read(), re.M)


def test_weights_and_topology_host_side():
    from tf_image_compression_amd.weights import synthetic_params, check_params, save_params, load_params
    from tf_image_compression_amd.topology import bottleneck_shape, layer_work
    p = synthetic_params(0)
    check_params(0, p)
    bad = dict(p)
    bad["encode_0/kernel"] = bad["encode_0/kernel"][..., :5]
    with pytest.raises(ValueError):
        check_params(0, bad)
    del bad["encode_0/kernel"]
    with pytest.raises(ValueError):
        check_params(0, bad)
    assert bottleneck_shape(0, 256) == (16, 16, 64)
    assert bottleneck_shape(3, 256) == (16, 16, 80)
    assert bottleneck_shape(3, 128) == (8, 8, 80)
    assert bottleneck_shape(2, 128) == (8, 8, 64)
    flops = sum(r[1] for r in layer_work(0, 256))
    assert abs(flops - 509.607936e6) < 1
    assert abs(sum(r[1] for r in layer_work(3, 256)) - 3878.682624e6) < 1


def test_npz_round_trip(tmp_path):
    from tf_image_compression_amd.weights import synthetic_params, save_params, load_params
    p = synthetic_params(2)
    save_params(str(tmp_path / "w.npz"), p)
    q = load_params(str(tmp_path / "w"))
    assert set(p) == set(q) and all(np.array_equal(p[k], q[k]) for k in p)


def test_bench_groups_fused_layer_pairs():
    """bench.py's roofline grouping: a layer launched inside the previous one (kernel name
    '') forms one group with it — FLOPs of both, the f32 intermediate excluded from bytes."""
    import importlib.util
    import os
    import numpy as np
    from tf_image_compression_amd.topology import layer_table, layer_work
    spec = importlib.util.spec_from_file_location("bench", os.path.join(os.path.dirname(__file__), "..", "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    L = len(layer_table(0))
    kernels = [f"k{i}" for i in range(L)]
    kernels[-1] = ""  # decode_0 inside decode_1's launch (dec10_kernel)
    groups, rows = bench.kernel_groups(None, 0, 256, np.full(L, 0.01), kernels)
    fused = [g for k, g in groups.items() if "fused" in k]
    assert len(fused) == 1 and fused[0]["layers"] == ["decode_1", "decode_0"] and fused[0]["launches"] == 1
    work = layer_work(0, 256)
    (l1, f1, b1, ho1), (l0, f0, b0, _) = work[-2], work[-1]
    assert fused[0]["flops"] == f1 + f0
    assert fused[0]["bytes"] == b1 + b0 - 2 * ho1 * ho1 * l1.cout * 4 == 64 * 64 * 32 * 4 + 256 * 256 * 3
    assert sum(g["launches"] for g in groups.values()) == L - 1


def test_bench_groups_chain_runs():
    """A wino_chain_kernel launch (encode_res_1/conv_0 .. encode_4 with the quantiser, and
    decode_4 .. decode_res_2/conv_1) is ONE group: the Winograd-form FLOPs of all five
    layers, HBM bytes = the first layer's f32 input + the last layer's output (u8 symbols on
    the encoder side), the step's rows counting every layer inside in the Winograd form."""
    import importlib.util
    import os
    import numpy as np
    from tf_image_compression_amd.topology import layer_table, layer_work
    spec = importlib.util.spec_from_file_location("bench", os.path.join(os.path.dirname(__file__), "..", "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    names = [lay.name for lay in layer_table(0)]
    L = len(names)
    kernels = [f"k{i}" for i in range(L)]
    e0, d0 = names.index("encode_res_1/conv_0"), names.index("decode_4")
    kernels[e0], kernels[d0] = "wino_chain_kernel<0,1,2>", "wino_chain_kernel<1,0,2>"
    for i in list(range(e0 + 1, e0 + 5)) + list(range(d0 + 1, d0 + 5)):
        kernels[i] = ""
    groups, rows = bench.kernel_groups(None, 0, 256, np.full(L, 0.01), kernels)
    chains = [g for g in groups.values() if len(g["layers"]) == 5]
    assert [g["layers"][0] for g in chains] == ["encode_res_1/conv_0", "decode_4"]
    work = layer_work(0, 256)
    for g, start in zip(chains, (e0, d0)):
        assert g["launches"] == 1
        assert g["flops"] == sum(work[i][1] for i in range(start, start + 5)) * bench.WINO_FRAC
    hw = 16 * 16 * 64
    assert chains[0]["bytes"] == hw * 4 + hw      # f32 in, u8 symbols out
    assert chains[1]["bytes"] == hw + hw * 4      # u8 symbols in, f32 out
    assert all(rows[i]["flops_per_patch"] == work[i][1] * bench.WINO_FRAC for i in range(e0, e0 + 5))
    assert sum(g["launches"] for g in groups.values()) == L - 8


def test_bench_dominant_by_kernel_family():
    """bench.py picks the dominant launch by kernel template over all its launches: the two
    chain runs (one template, two instances) are one family whose one-lane time is their sum,
    so a 50.6 / 50.3 us tie between them cannot flip the pick; the family's roofline is the
    mean FLOPs per launch over the mean duration."""
    import importlib.util
    import os
    import numpy as np
    from tf_image_compression_amd.topology import layer_table
    spec = importlib.util.spec_from_file_location("bench", os.path.join(os.path.dirname(__file__), "..", "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    lt = layer_table(0)
    names = {lay.name: i for i, lay in enumerate(lt)}
    L = len(lt)
    kernels = [f"k{i}_kernel<{i}>" for i in range(L)]
    kernels[2], kernels[3] = "conv3x3_kernel<2,32>", "conv3x3_kernel<2,64>"
    e0, d0 = names["encode_res_1/conv_0"], names["decode_4"]
    kernels[e0], kernels[d0] = "wino_chain_kernel<0,1,2>", "wino_chain_kernel<1,0,2>"
    for i in list(range(e0 + 1, e0 + 5)) + list(range(d0 + 1, d0 + 5)):
        kernels[i] = ""
    ms = np.full(L, 0.02)
    ms[0] = 0.0506  # a single launch slower than either chain launch
    ms[e0], ms[d0] = 0.0503, 0.0501
    groups, _ = bench.kernel_groups(None, 0, 256, ms, kernels)
    fams = bench.kernel_families(groups, kernels, names)
    dom = max(fams, key=lambda f: (fams[f]["ms"], fams[f]["flops"]))
    assert dom == "wino_chain_kernel" and fams[dom]["launches"] == 2 and len(fams[dom]["members"]) == 2
    f = fams[dom]
    gs = [groups[k] for k in f["members"]]
    roof, ms_launch, flops, _ = bench.roofline_of(f, 32)
    assert abs(ms_launch - (0.0503 + 0.0501) / 2) < 1e-12
    assert abs(flops - 32 * (gs[0]["flops"] + gs[1]["flops"]) / 2) < 1e-3
    # two instances of another template are one family too (the template name up to '<')
    assert fams["conv3x3_kernel"]["launches"] == 2 and len(fams) == L - 10


def test_bench_groups_chain_with_stride2_neighbours():
    """With chain_x the encoder chain launch starts at encode_3 (its stride-2 head) and the
    decoder chain launch ends with decode_3 and decode_2: one group each, whose FLOPs count the
    Winograd form only for the stride-1 layers and the direct form for the stride-2 /
    transposed ones (bench.kernel_groups), HBM bytes = the head's f32 input + the u8 symbols,
    and the symbols + decode_2's f32 output."""
    import importlib.util
    import os
    import numpy as np
    from tf_image_compression_amd.topology import layer_table, layer_work
    spec = importlib.util.spec_from_file_location("bench", os.path.join(os.path.dirname(__file__), "..", "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    lt = layer_table(0)
    names = [lay.name for lay in lt]
    L = len(names)
    kernels = [f"k{i}" for i in range(L)]
    e3, d0, d2 = names.index("encode_3"), names.index("decode_4"), names.index("decode_2")
    kernels[e3], kernels[d0] = "wino_chain_kernel<0,1,2,1>", "wino_chain_kernel<1,0,2,6>"
    for i in list(range(e3 + 1, e3 + 6)) + list(range(d0 + 1, d2 + 1)):
        kernels[i] = ""
    groups, rows = bench.kernel_groups(None, 0, 256, np.full(L, 0.01), kernels)
    enc = next(g for g in groups.values() if g["layers"][0] == "encode_3")
    dec = next(g for g in groups.values() if g["layers"][0] == "decode_4")
    assert enc["layers"][-1] == "encode_4" and dec["layers"][-1] == "decode_2"
    work = layer_work(0, 256)
    frac = lambda i: bench.WINO_FRAC if lt[i].kind == "conv_s1" else 1.0
    assert enc["flops"] == sum(work[i][1] * frac(i) for i in range(e3, e3 + 6))
    assert dec["flops"] == sum(work[i][1] * frac(i) for i in range(d0, d2 + 1))
    assert rows[e3]["flops_per_patch"] == work[e3][1]  # the head: direct
    assert enc["bytes"] == 32 * 32 * 64 * 4 + 16 * 16 * 64
    assert dec["bytes"] == 16 * 16 * 64 + 64 * 64 * 32 * 4


def test_bench_direct_equiv_mixed_form_chain():
    """roofline.direct_equiv_tflops of the chain family with its stride-2 head and transposed
    tail: only the Winograd layers are converted to the direct form.  With
    round 5's one-lane launch times (55.72 / 75.84 us per 32-patch launch) the direct-form
    work (3.623 + 4.831 GFLOP) over 131.56 us is 64.3 TF/s, not the 87.2 that dividing the
    whole group by 16/36 gave; `frac` stays on the executed (minimal-form) FLOPs."""
    import importlib.util
    import os
    import numpy as np
    from tf_image_compression_amd.topology import layer_table, layer_work
    spec = importlib.util.spec_from_file_location("bench", os.path.join(os.path.dirname(__file__), "..", "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    lt = layer_table(0)
    names = {lay.name: i for i, lay in enumerate(lt)}
    L = len(lt)
    kernels = [f"k{i}" for i in range(L)]
    e3, d0, d2 = names["encode_3"], names["decode_4"], names["decode_2"]
    kernels[e3], kernels[d0] = "wino_chain_kernel<0,1,2,1>", "wino_chain_kernel<1,0,2,6>"
    for i in list(range(e3 + 1, e3 + 6)) + list(range(d0 + 1, d2 + 1)):
        kernels[i] = ""
    ms = np.full(L, 0.001)
    ms[e3], ms[d0] = 0.05572, 0.07584
    groups, _ = bench.kernel_groups(None, 0, 256, ms, kernels)
    fams = bench.kernel_families(groups, kernels, names)
    fam = fams["wino_chain_kernel"]
    work = layer_work(0, 256)
    direct = sum(work[i][1] for i in range(e3, e3 + 6)) + sum(work[i][1] for i in range(d0, d2 + 1))
    assert abs(fam["direct_flops"] * 2 - direct) < 1e-3
    roof, dom_ms, dom_flops, _ = bench.roofline_of(fam, 32)
    dom_k = sorted({kernels[names[nm]] for nm in fam["layers"]} - {""})
    bench.winograd_note(roof, dom_k, fam, 32, dom_ms)
    assert abs(direct * 32 / 1e9 - (3.623 + 4.831)) < 0.01
    assert abs(roof["direct_equiv_tflops"] - 64.3) < 0.1, roof
    assert "stride-2 / transposed ones in their own form" in roof["flop_form"]
    assert abs(roof["frac"] - 0.2465) < 0.002  # executed FLOPs over the peak, unchanged
    # the decoder chain with its decode_2 in the polyphase form (HT bit 8): that layer counts
    # 25/36 of its direct FLOPs, the rest as before
    kernels[d0] = "wino_chain_kernel<1,0,2,14>"
    groups14, _ = bench.kernel_groups(None, 0, 256, ms, kernels)
    fam14 = bench.kernel_families(groups14, kernels, names)["wino_chain_kernel"]
    assert abs(fam14["direct_flops"] - fam["direct_flops"]) < 1e-6
    assert abs((fam["flops"] - fam14["flops"]) * 2 - work[d2][1] * (1 - bench.PWINO_FRAC)) < 1e-3
    # a pure Winograd group keeps the plain 16/36 conversion
    g = {"flops": 10e9 * bench.WINO_FRAC, "direct_flops": 10e9}
    r = {}
    bench.winograd_note(r, ["conv3x3_wino_kernel<64,64>"], g, 1, 1.0)
    assert r["direct_equiv_tflops"] == 10.0 and "stride-2" not in r["flop_form"]
