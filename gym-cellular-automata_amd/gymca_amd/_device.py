"""Device plumbing: torch tensors as HBM buffers, the current HIP stream, H2D/D2H moves.

PyTorch is used only for device memory, streams and torch.distributed; every byte of
CA arithmetic happens in libgca_hip.so.
"""
import numpy as np

from ._lib import GCAError

try:
    import torch
except ImportError:  # pragma: no cover
    torch = None


def require_device(device=None):
    """Return a torch.device for the GPU or raise: the product path has no CPU fallback."""
    if torch is None or not torch.cuda.is_available():
        raise GCAError("gymca_amd needs a HIP device (MI355X); none is visible in this process")
    if device is None:
        return torch.device("cuda", torch.cuda.current_device())
    device = torch.device(device)
    if device.type != "cuda":
        raise GCAError(f"gymca_amd runs on the GPU only, got device {device}")
    return device


def is_device_tensor(x):
    return torch is not None and isinstance(x, torch.Tensor) and x.is_cuda


def device_index(device=None):
    if device is None:
        return torch.cuda.current_device()
    if isinstance(device, int):
        return device
    device = torch.device(device)
    return device.index if device.index is not None else torch.cuda.current_device()


def stream_ptr(device=None):
    """The raw hipStream_t of the current stream on `device` (torch's work and hipGraph capture order with it).
    torch.cuda.current_stream(device).cuda_stream builds a Stream object per call; the raw accessor is the same value
    at a fraction of the host cost (the batched envs call it on every step)."""
    return raw_stream(device_index(device))


def raw_stream(index):
    """stream_ptr for a known device index (no device parsing)."""
    return torch._C._cuda_getCurrentRawStream(index)


def ptr(t):
    """Device address of a contiguous CUDA tensor (None -> NULL)."""
    if t is None:
        return None
    if not (t.is_cuda and t.is_contiguous()):
        raise GCAError("expected a contiguous device tensor")
    return t.data_ptr()


def to_device(x, dtype, device):
    """numpy / tensor -> contiguous device tensor of `dtype` (a torch dtype)."""
    if is_device_tensor(x):
        return x.to(device=device, dtype=dtype).contiguous()
    arr = np.ascontiguousarray(np.asarray(x))
    return torch.from_numpy(arr).to(device=device, dtype=dtype, non_blocking=False).contiguous()


def check_u8_codes(values):
    for v in values:
        if not (0 <= int(v) <= 255):
            raise ValueError(f"cell value {v} does not fit the u8 device layout (0..255)")
