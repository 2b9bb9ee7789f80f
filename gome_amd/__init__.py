"""gome_amd: MI355X batch matching engine (libgome.so behind include/gome/gome_abi.h)."""
import os

# The engine runs a batch on five HIP streams.  HIP maps streams onto at most
# GPU_MAX_HW_QUEUES hardware queues per process (default 4) and streams that share a queue run
# one after another, so the engine asks for 16 (room for torch's and RCCL's streams beside its
# own) when the package is imported before the HIP runtime starts (the runtime reads the variable
# once, at its initialisation; never lowered, at most 32).
# libgome.so checks the same variable and keeps the old four-stream layout when it is below 8.
if os.environ.get("GOME_HW_QUEUES"):  # (an exact value, for A/B)
    os.environ["GPU_MAX_HW_QUEUES"] = os.environ["GOME_HW_QUEUES"]
elif int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or "4") < 16:
    os.environ["GPU_MAX_HW_QUEUES"] = "16"
