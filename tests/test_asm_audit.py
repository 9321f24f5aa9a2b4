"""CPU: the inline-asm clobber audit (tools/asm_audit.py) over every device
translation unit -- each implicit VCC / SCC / EXEC write of an asm template
is declared (the round-2 hang came from an undeclared SCC write) -- and the
auditor itself catches such a template."""
import os
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tools"))
import asm_audit  # noqa: E402


def test_every_asm_statement_declares_its_implicit_writes():
    if not os.path.exists("/opt/rocm/bin/hipcc"):
        pytest.skip("hipcc not present")
    total, bad = 0, []
    for f in asm_audit.sources():
        n, issues = asm_audit.audit(f)
        total += n
        bad += issues
    assert total >= 100  # the field/scalar/SHA carry chains, rare folds, DPP rows
    assert not bad, bad


def test_auditor_flags_undeclared_writes(tmp_path):
    assert asm_audit.writes("v_add_co_u32_e32 %0, vcc, %0, %1") == {"vcc"}
    assert asm_audit.writes("s_or_b64 %0, %1, %2") == {"scc"}
    assert asm_audit.writes("s_and_saveexec_b64 %0, %1") == {"exec", "scc"}
    assert asm_audit.writes("v_mad_u64_u32 %0, %1, %2, %3, %4") == set()
    assert asm_audit.writes("s_nop 1\n\ts_cbranch_vccz 1f\n1:") == set()
    if not os.path.exists("/opt/rocm/bin/hipcc"):
        return
    src = tmp_path / "bad.hip"
    src.write_text('#include <hip/hip_runtime.h>\n'
                   '__global__ void k(unsigned* o, unsigned long long a) {\n'
                   '  unsigned long long r;\n'
                   '  asm volatile("s_or_b64 %0, %1, %1" : "=s"(r) : "s"(a));\n'
                   '  unsigned c = o[0];\n'
                   '  asm volatile("v_add_co_u32_e32 %0, vcc, %0, %0" : "+v"(c) : : "vcc");\n'
                   '  o[0] = c + (unsigned)r;\n}\n')
    n, issues = asm_audit.audit(str(src))
    assert n >= 2 and len(issues) == 1 and "scc" in issues[0], issues
