"""CPU check of the PyTorch engine's single-arena layout
(models/torch_kiosk.py): the carver hands out aligned, non-overlapping
typed views, and the size the engine reserves for the weights is exactly
what :func:`ops.kernels.model_weights` takes from it."""
import json
import os
import subprocess
import sys

import pytest

torch = pytest.importorskip('torch')


def test_carver_views_are_aligned_and_disjoint():
    from kiosk_autoscaler_amd.models import torch_kiosk as tk
    specs = [('a', (3,), torch.float32), ('b', (5, 7), torch.bfloat16),
             ('c', (1,), torch.int64), ('d', (64, 2), torch.int32)]
    arena = torch.zeros(tk._span(specs), dtype=torch.uint8)
    carve = tk._Carver(arena)
    views = [carve(shape, dtype) for _, shape, dtype in specs]
    assert carve.offset == arena.numel()
    base = arena.data_ptr()
    spans = []
    for view, (_, shape, dtype) in zip(views, specs):
        assert tuple(view.shape) == shape and view.dtype == dtype
        start = view.data_ptr() - base
        assert start % 256 == 0
        spans.append((start, start + view.numel() * view.element_size()))
    for (s0, e0), (s1, _) in zip(spans, spans[1:]):
        assert e0 <= s1
    views[1].fill_(1.5)
    assert float(views[0].sum()) == 0 and float(views[2].sum()) == 0
    with pytest.raises(RuntimeError):
        carve((1,), torch.float32)


def test_weight_reservation_matches_model_weights_allocation():
    """model_weights asks its allocator for w1, b1, w2, b2 per layer before
    it launches anything: the engine's reservation is their aligned sum."""
    from kiosk_autoscaler_amd.models import torch_kiosk as tk
    from kiosk_autoscaler_amd.ops import kernels
    dim, hidden = 64, 256
    order = []

    class Sized(Exception):
        pass

    def record(shape, dtype):
        order.append((tuple(shape), dtype))
        if len(order) == 4:
            raise Sized()
        return None
    with pytest.raises(Sized):
        kernels.model_weights(dim, hidden, 1, 7, alloc=record)
    assert order == [((hidden, dim), torch.bfloat16),
                     ((hidden,), torch.float32),
                     ((dim, hidden), torch.bfloat16),
                     ((dim,), torch.float32)]
    size = sum(tk._aligned(tk._nbytes(s, d)) for s, d in order)
    assert size == tk._layer_bytes(dim, hidden)


def test_rocm_comgr_replaces_torchs_bundled_copy():
    """``native.prefer_rocm_comgr`` before ``import torch``: one comgr is
    mapped, ROCm's, and torch's HIP runtime is still torch's own (no second
    HIP runtime).  After torch is imported it is a no-op."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    child = (
        'import json, sys\n'
        'sys.path.insert(0, sys.argv[1])\n'
        'from kiosk_autoscaler_amd.ops import native\n'
        'first = native.prefer_rocm_comgr()\n'
        'import torch\n'
        'again = native.prefer_rocm_comgr()\n'
        'maps = [l.split()[-1] for l in open("/proc/self/maps")]\n'
        'print(json.dumps({"first": first, "again": again,\n'
        '  "comgr": sorted({m for m in maps if "comgr" in m}),\n'
        '  "hip": sorted({m for m in maps if "libamdhip64" in m})}))\n')
    out = subprocess.run([sys.executable, '-c', child, root],
                         stdout=subprocess.PIPE, timeout=300, check=True)
    row = json.loads(out.stdout.decode().strip().splitlines()[-1])
    if row['first'] is None:
        pytest.skip('no ROCm comgr in the loader cache')
    assert row['comgr'] == [row['first']]
    assert row['first'].startswith('/opt/rocm')
    assert row['again'] is None
    assert len(row['hip']) == 1 and 'torch' in row['hip'][0]


def test_bundled_comgr_opt_out(monkeypatch):
    from kiosk_autoscaler_amd.ops import native
    monkeypatch.setenv('KIOSK_TORCH_COMGR', 'bundled')
    monkeypatch.delitem(sys.modules, 'torch', raising=False)
    assert native.prefer_rocm_comgr() is None


def test_rocm_comgr_preferred_only_with_torchs_abi(tmp_path):
    """ROCm's comgr replaces torch's bundled copy only when both
    carry the same soname (comgr ABI major) -- another ROCm / torch pair
    keeps the bundled one."""
    import subprocess
    from kiosk_autoscaler_amd.ops import native
    src = tmp_path / 'c.c'
    src.write_text('int amd_comgr_x(void) { return 3; }\n')

    def lib(name, soname):
        out = tmp_path / name
        subprocess.run(['gcc', '-shared', '-fPIC', str(src), '-o', str(out),
                        '-Wl,-soname,' + soname], check=True)
        return str(out)
    rocm3 = lib('rocm3.so', 'libamd_comgr.so.3')
    torch3 = lib('torch3.so', 'libamd_comgr.so.3')
    torch2 = lib('torch2.so', 'libamd_comgr.so.2')
    assert native.elf_soname(rocm3) == 'libamd_comgr.so.3'
    assert native.comgr_abi_matches(torch_lib=torch3, rocm_lib=rocm3)
    assert not native.comgr_abi_matches(torch_lib=torch2, rocm_lib=rocm3)
    assert not native.comgr_abi_matches(torch_lib=str(tmp_path / 'none'),
                                        rocm_lib=rocm3)
