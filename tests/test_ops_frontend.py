"""CPU checks of the torch front end of the native kernels (``ops/``): the
loader's loud failure, and argument validation that must reject a bad call
*before* anything reaches a kernel launch (a wrong shape or a host pointer
handed to a gfx950 kernel faults the device, not Python).  The launches
themselves are GPU tests (``test_gpu_kernels.py``)."""
import pytest

torch = pytest.importorskip('torch')

from kiosk_autoscaler_amd.ops import kernels, native  # noqa: E402


def _built():
    return bool(native.extension_candidates())


def test_loader_fails_loudly_without_the_extension(monkeypatch):
    monkeypatch.setattr(native, '_MOD', None)
    monkeypatch.setattr(native, 'extension_candidates', lambda: [])
    with pytest.raises(native.NativeUnavailable) as err:
        native.load()
    assert 'tools/build_native.py' in str(err.value)
    assert native.available() is False


def test_loader_reports_an_unimportable_extension(monkeypatch):
    import importlib
    monkeypatch.setattr(native, '_MOD', None)
    monkeypatch.setattr(native, 'extension_candidates', lambda: ['x.so'])

    def broken(name):
        raise ImportError('undefined symbol: hipFoo')
    monkeypatch.setattr(importlib, 'import_module', broken)
    with pytest.raises(native.NativeUnavailable) as err:
        native.load(torch_first=False)
    assert 'hipFoo' in str(err.value) and 'build_native' in str(err.value)


@pytest.mark.skipif(not _built(), reason='extension not built')
def test_loaded_module_is_the_in_tree_gfx950_build():
    mod = native.load()
    assert mod.arch == 'gfx950'
    assert native.loaded_path().startswith(native.HERE)
    assert native.available()


@pytest.mark.skipif(not _built(), reason='extension not built')
def test_gemm_rejects_bad_operands_before_launch():
    a = torch.zeros(256, 128, dtype=torch.bfloat16)       # host tensor
    with pytest.raises(ValueError, match='CUDA tensor'):
        kernels.gemm(a, a)
    with pytest.raises(ValueError, match='CUDA tensor'):
        kernels.gemm(a.float(), a)
    with pytest.raises(ValueError, match='CUDA tensor'):
        kernels.gemm(a.t(), a)                            # not contiguous


@pytest.mark.skipif(not _built(), reason='extension not built')
def test_init_and_checksum_reject_host_tensors():
    with pytest.raises(ValueError, match='GPU'):
        kernels.init_uniform_(torch.zeros(16), 1)
    with pytest.raises(ValueError, match='CUDA tensor'):
        kernels.checksum(torch.zeros(16, dtype=torch.bfloat16))


def test_reference_forward_keeps_the_kernels_bf16_storage_points():
    """The fp32 reference rounds the hidden activation and every layer's
    output to bf16, exactly where the kernels store them."""
    from kiosk_autoscaler_amd.models.mlp import GELU_C
    g = torch.Generator().manual_seed(3)
    dim, hidden, rows = 32, 64, 8

    def rnd(*shape, dtype=torch.bfloat16, scale=0.2):
        return (torch.rand(*shape, generator=g) * 2 - 1).mul(scale).to(dtype)
    weights = [(rnd(hidden, dim), rnd(hidden, dtype=torch.float32),
                rnd(dim, hidden), rnd(dim, dtype=torch.float32))
               for _ in range(2)]
    x = rnd(rows, dim, scale=1.0)
    got = kernels.reference_forward(x, weights)
    assert got.dtype == torch.bfloat16 and tuple(got.shape) == (rows, dim)
    ref = x
    for w1, b1, w2, b2 in weights:
        h = ref.float() @ w1.float().t() + b1
        h = 0.5 * h * (1 + torch.tanh(GELU_C * (h + 0.044715 * h ** 3)))
        h = h.to(torch.bfloat16).float()
        ref = (h @ w2.float().t() + b2 + ref.float()).to(torch.bfloat16)
    torch.testing.assert_close(got, ref, rtol=0, atol=0)
