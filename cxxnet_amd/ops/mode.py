"""Precision mode of the GPU executor.

bf16 (default): activations bf16, every op on the HIP kernels (fp32 accumulation, fp32 master
weights and optimizer state).  fp32 ("precision = fp32" in a conf, or set_reference_precision):
the GPU runs the executor's fp32 reference formulas -- the torch code the CPU path uses -- on
device tensors, the reference's own precision (cxxnet's real_t = float).  It is a parity oracle
at production batch sizes (tests/test_fp32_mode_gpu.py compares the bf16 kernels against it on
the real AlexNet graph), not a fast path."""
import torch

_REF = {"on": False}


def set_reference_precision(on: bool = True):
    _REF["on"] = bool(on)


def reference_precision() -> bool:
    return _REF["on"]


def native(t: torch.Tensor) -> bool:
    """Whether an op on tensor t runs its HIP kernel (GPU tensor, bf16 mode)."""
    return t.is_cuda and not _REF["on"]


_REC = {"on": False}


def set_recording(on: bool):
    """A C++ launch list is being recorded (NetTrainer._list_step)."""
    _REC["on"] = bool(on)


def frozen() -> bool:
    """The step's launches are being frozen for replay -- recorded into a C++ launch list or
    captured into a HIP graph: no autotuning launches, no side streams, no host reads."""
    return _REC["on"] or torch.cuda.is_current_stream_capturing()


# Buffers a recorded launch list or captured HIP graph may still point at.  A module-level
# workspace that grows is replaced, and a replay of a step recorded before the growth would write
# into the freed block -- which the caching allocator may have handed to a live tensor by then
# (round 4: a step recorded while the unfused fc weight-grad grew the split-K workspace replayed
# its earlier partial sums into the next batch's input).  Replaced workspaces are retired here
# instead of freed; they only grow, so this holds less than the final size again.
_GRAVE = []


def retire(t):
    """Keep a replaced workspace alive for the plans that may still reference it."""
    if t is not None:
        _GRAVE.append(t)
