"""CPU check of the PyTorch engine's single-arena layout
(models/torch_kiosk.py): the carver hands out aligned, non-overlapping
typed views, and the size the engine reserves for the weights is exactly
what :func:`ops.kernels.model_weights` takes from it."""
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
