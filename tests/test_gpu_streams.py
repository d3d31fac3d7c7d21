"""Side streams that run beside the caller's (ops.concurrent_stream): a pooled torch stream may share the caller's
hardware queue (GPU_MAX_HW_QUEUES), which serialises a trainer's side-stream work behind its main chain (kernel
traces: DESIGN §3.9).  The probe (vm_spin on the caller's stream, a short kernel on the candidate) must pick a stream
whose kernels finish while the caller's stream is still busy, and the UNetImage trainer must use it."""

import pytest
import torch

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a ROCm GPU")]


def test_concurrent_stream_runs_beside_the_caller():
    from vmatting import ops
    dev = torch.device("cuda", 0)
    s = ops.concurrent_stream(dev)
    assert s is ops.concurrent_stream(dev)  # cached per (device, caller stream)
    main = torch.cuda.current_stream(dev)
    assert s.cuda_stream != main.cuda_stream
    assert all(ops._runs_beside(main, s) for _ in range(3))


def test_spin_holds_the_stream():
    """vm_spin(us) keeps its stream busy for about that long (the probe's premise)."""
    import ctypes
    import time
    from vmatting import _lib
    st = torch.cuda.current_stream()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    _lib.check(_lib.lib().vm_spin(20000, ctypes.c_void_p(st.cuda_stream)), "spin")
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    assert 0.015 <= dt <= 0.5, dt


def test_image_trainer_side_stream_is_probed():
    from oracle.models import synthetic_vgg16
    from vmatting import ops
    from vmatting.image_train import ImageTrainer
    dev = torch.device("cuda", 0)
    trn = ImageTrainer(synthetic_vgg16(0), "bf16", dev)
    assert ImageTrainer.side_kind == "probe"
    assert trn._side is ops.concurrent_stream(dev)
