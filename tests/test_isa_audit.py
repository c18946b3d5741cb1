"""The built library holds no packed-fp32 VALU op that swaps a source operand's 32-bit halves (op_sel 1 with
op_sel_hi 0 on the same source): on MI355X that form intermittently produced wrong lanes 48-63 under concurrent
kernels (tools/pk_bisect.py).  styletts-zs_amd/build.py compiles the files where hipcc emitted it
without packed-fp32 ops; this audit disassembles every gfx950 code object of libstzs_hip.so (CPU only: no GPU call)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "styletts-zs_amd", "stzs", "libstzs_hip.so")


@pytest.mark.skipif(not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-objdump") or not os.path.exists(LIB),
                    reason="needs the ROCm llvm-objdump and the built library")
def test_no_swapped_packed_fp32_operands():
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import pk_audit
    res = pk_audit.audit(LIB)
    assert res, "no kernel disassembled"
    bad = {k: v["swap"] for k, v in res.items() if v.get("swap", 0)}
    assert not bad, f"kernels with swapped-operand packed-fp32 ops: {bad}"
    print("kernels with packed-fp32 ops:", len(res), "| swapped-operand ops: 0")
