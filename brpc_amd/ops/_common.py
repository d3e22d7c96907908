import torch

from ..native import native


def stream_handle(device=None):
    return torch.cuda.current_stream(device).cuda_stream


def require_gpu_tensor(t, name="tensor"):
    if not isinstance(t, torch.Tensor):
        raise TypeError("%s must be a torch.Tensor" % name)
    if not t.is_cuda:
        raise ValueError("%s must live on a GPU (got %s)" % (name, t.device))
    if not t.is_contiguous():
        raise ValueError("%s must be contiguous" % name)
    if native.gpu.device_count() <= 0:
        raise RuntimeError("brpc_amd native runtime sees no HIP device")


def nbytes(t):
    return t.numel() * t.element_size()
