#!/usr/bin/env python3
"""Run only the Inception branch-3 pool backward at the 3b shape (for rocprofv3 --pmc passes).

    python tools/pool_probe.py [impl]      impl 1 = LDS scatter (default), 0 = sliding gather
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from mil_nce_howto100m_amd.ops import hip_ops as h  # noqa: E402
from mil_nce_howto100m_amd.ops._lib import lib  # noqa: E402

impl = int(sys.argv[1]) if len(sys.argv) > 1 else 1
lib().milnce_set_pool_s1_impl(impl)
x = torch.randn(256, 8, 25, 25, 192, device="cuda").to(torch.bfloat16).requires_grad_(True)
dy = torch.randn(256, 8, 25, 25, 192, device="cuda").to(torch.bfloat16)
y = h.maxpool3d(x, (3, 3, 3), (1, 1, 1), False)
for _ in range(3):
    torch.autograd.grad(y, x, dy, retain_graph=True)
torch.cuda.synchronize()
print("done")
