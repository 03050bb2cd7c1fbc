#!/usr/bin/env python3
"""List the ATen compute kernels left on a model's GPU path (no GPU needed).

Runs the same meta-device forward passes as ``arbius_amd.ops.audit`` (HIP launches recorded, not
executed) under a TorchDispatchMode that records every ATen op which would launch a device kernel
(views, allocations and metadata ops excluded), with the model source line that issued it:

    python scripts/aten_audit.py sd15 512 4
    python scripts/aten_audit.py kandinsky2 768 4
    python scripts/aten_audit.py zeroscopev2xl 576 1 24      (width; height = width * 320 / 576)
"""
import collections
import os
import sys
import traceback

from torch.utils._python_dispatch import TorchDispatchMode

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from arbius_amd.ops import audit  # noqa: E402

# ops that never launch a kernel (views / allocation / metadata)
_FREE = {
    "empty", "empty_like", "empty_strided", "new_empty", "new_empty_strided", "view", "_unsafe_view", "reshape",
    "as_strided", "t", "transpose", "permute", "expand", "unsqueeze", "squeeze", "slice", "select", "split",
    "split_with_sizes", "chunk", "unbind", "detach", "alias", "lift_fresh", "_to_copy_meta", "unflatten",
    "flatten", "view_as", "narrow", "movedim", "expand_as", "_reshape_alias", "diagonal", "sym_size",
    "is_same_size", "_has_compatible_shallow_copy_type", "set_", "resize_", "contiguous_meta",
    "_local_scalar_dense", "item", "dim", "size", "stride", "numel", "is_contiguous", "clone_meta",
}


# module construction and the derived-weight caches (computed once per live weight, ops.derived_ready)
_ONCE = {"__init__", "_build", "ln_fold", "_padded_weights", "interleave_geglu", "_cached_weights", "_fused_weights"}


class _Rec(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.hits = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = func.overloadpacket.__name__
        out = func(*args, **(kwargs or {}))
        if name not in _FREE and not name.startswith("_foreach"):
            stack = traceback.extract_stack()[:-1]
            if any(fr.name in _ONCE for fr in stack):
                return out          # module construction / cached weight derivations, not per step
            where = "?"
            for fr in reversed(stack):
                if "/arbius_amd/" in fr.filename and "/ops/" not in fr.filename:
                    where = f"{fr.filename.split('/arbius_amd/')[1]}:{fr.lineno}"
                    break
            self.hits[(name, where)] += 1
        return out


def main():
    model = sys.argv[1] if len(sys.argv) > 1 else "sd15"
    size = int(sys.argv[2]) if len(sys.argv) > 2 else 512
    group = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    frames = int(sys.argv[4]) if len(sys.argv) > 4 else 24
    fn = {"sd15": audit.sd15, "kandinsky2": audit.kandinsky2,
          "zeroscopev2xl": lambda w, h, g: audit.video("zeroscopev2xl", w, h, frames),
          "damo": lambda w, h, g: audit.video("damo", w, h, frames)}[model]
    rec = _Rec()
    with rec:
        fn(size, size * 320 // 576 if model == "zeroscopev2xl" else size, group)
    total = sum(rec.hits.values())
    print(f"{model} {size}^2 group {group}: {total} ATen kernel launches outside the HIP ops")
    for (name, where), n in rec.hits.most_common():
        print(f"{n:6d}  {name:28s} {where}")


if __name__ == "__main__":
    main()
