"""Static determinism guards over the HIP sources (SURVEY.md §5.2 race detection / §7.3.1).

A solution CID is consensus, so no floating-point reduction may depend on arrival order: every
kernel reduces in a fixed order (LDS trees, xor butterflies, ordered split-K slabs).  The one
atomics in the kernel library are integer TICKETS: the split-K ticket (which block of a tile reduces
the slabs - the reduction itself still walks slabs 0..S-1 in order) and the GroupNorm stats ticket
(which block of an image builds the table - from the partials in the fixed tree order of the table
kernel); anything else fails here.
"""
import os
import re

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "arbius_amd", "ops", "csrc")
ATOMIC = re.compile(r"\b(atomicAdd|atomicCAS|atomicExch|atomicMax|atomicMin|unsafeAtomicAdd|__hip_atomic_\w+|"
                    r"global_atomic_\w+|buffer_atomic_\w+|ds_add_\w+|__atomic_\w+)\b")
ALLOWED = {("conv.hip", "__hip_atomic_fetch_add"),      # integer split-K ticket, ordered slab reduce
           ("groupnorm.hip", "__hip_atomic_fetch_add")}  # integer stats ticket, fixed-tree table


def _code_lines(path):
    """Source lines with // comments stripped (the sources document 'no atomics' in comments)."""
    for i, line in enumerate(open(path), 1):
        yield i, line.split("//", 1)[0]


def test_no_float_atomics_in_kernels():
    found = []
    for name in sorted(os.listdir(CSRC)):
        if not name.endswith((".hip", ".h", ".inc")):
            continue
        for i, code in _code_lines(os.path.join(CSRC, name)):
            for m in ATOMIC.finditer(code):
                if (name, m.group(1)) not in ALLOWED:
                    found.append(f"{name}:{i}: {m.group(1)}")
    assert not found, "order-dependent atomics in the kernel library: " + ", ".join(found)


def test_split_k_ticket_is_integer_and_reduction_is_ordered():
    src = open(os.path.join(CSRC, "conv.hip")).read()
    calls = re.findall(r"__hip_atomic_fetch_add\(([^;]*)\);", src)
    assert len(calls) == 1 and "counters" in calls[0]            # int* ticket pool, never a float slab
    # the reducer sums slabs sp = 1 .. nsplit-1 in index order onto slab 0
    assert re.search(r"for \(int sp = 1; sp < p\.nsplit; \+\+sp\)", src)


def test_group_norm_ticket_is_integer_and_table_tree_is_shared():
    src = open(os.path.join(CSRC, "groupnorm.hip")).read()
    calls = re.findall(r"__hip_atomic_fetch_add\(([^;]*)\);", src)
    assert len(calls) == 1 and "tickets" in calls[0]             # int* ticket per image
    # the last block builds the table with the table kernel's own tree (one definition, two callers)
    assert src.count("gn_table_tree(") == 3                        # definition + wave kernel + fused tail
