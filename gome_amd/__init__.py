"""gome_amd: MI355X batch matching engine (libgome.so behind include/gome/gome_abi.h)."""
import os
import sys

# The engine runs a batch on five HIP streams.  HIP maps streams onto at most
# GPU_MAX_HW_QUEUES hardware queues per process (default 4), and streams that share a queue run
# one after another.  So the package asks for 16 (room for torch's and RCCL's streams beside the
# engine's own) when it is imported before the HIP runtime starts: the runtime reads the variable
# once, when it initialises.  It never lowers the variable (the pool allows at most 32).
# What the runtime will actually have is recorded in _HW_QUEUES and passed to every engine as
# gome_config.hw_queues, which picks the stream layout.  The library does not guess it from the
# environment: the variable may have changed after HIP started.


def _parse_queues(v):
    try:
        q = int(str(v).strip())
    except (TypeError, ValueError):
        return None
    return q if 0 < q < 1024 else None


def _hip_started() -> bool:
    """True when a HIP runtime in this process has (as far as we can tell) already initialised:
    torch's, the only other HIP user the package knows of."""
    torch = sys.modules.get("torch")
    try:
        return bool(torch is not None and torch.cuda.is_initialized())
    except Exception:  # pragma: no cover
        return False


_env = _parse_queues(os.environ.get("GPU_MAX_HW_QUEUES"))
if _hip_started():
    _HW_QUEUES = _env or 4  # (too late to change: the runtime kept what it read)
else:
    _want = _parse_queues(os.environ.get("GOME_HW_QUEUES"))  # (an exact value, for A/B)
    if _want is None:
        _want = max(_env or 4, 16)
    os.environ["GPU_MAX_HW_QUEUES"] = str(_want)
    _HW_QUEUES = _want


def hw_queues() -> int:
    """The hardware queues the process's HIP runtime has (or will have when it starts)."""
    return _HW_QUEUES
