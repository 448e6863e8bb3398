"""oracle/ — TEST INFRASTRUCTURE ONLY. CPU restatement of the reference's YOLOv7 inference path.

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import anything
from here, and only as the checker / the timed CPU baseline — never as part of the product path.

Parity status:
  * Graph structure: PINNED — the cfg dicts the product generates are compared with the reference
    YAML files (tests/test_arch.py) whenever /root/reference is present.
  * NMS / decode semantics: PINNED BY HAND-DERIVED KNOWN-ANSWER CASES (tests/test_oracle_kat.py);
    torchvision.ops.nms itself is an un-vendored third-party dependency with no pinned version
    in the reference, restated here from its published algorithm.
  * Conv / activation numerics: PARITY UNPINNED — the reference has no tests, no golden vectors
    and no weights, and importing/running it in this container was denied.  The
    restatement calls the same ATen CPU ops (F.conv2d, F.silu, F.leaky_relu, F.max_pool2d,
    torch.cat, F.interpolate) in the reference's order, so on the same torch build it reproduces
    the reference CPU path op for op, but no reference-produced vector pins it.
"""
