"""The hand-counted `s_waitcnt vmcnt(N)` after inline-asm loads in the rx hot
path, checked on the emitted gfx950 ISA: on every
control-flow path no instruction names an in-flight load's destination
registers before a wait that covers it, and each asm block's covering asm
wait counts exactly the vector-memory instructions issued since (tests/
isa_check.py).  The check must also fail on deliberately perturbed builds:
an extra load between a slot read and its wait (USN_ISA_PERTURB=1), and a
stale count (=2)."""
import os

import pytest

import isa_check

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "usnetd_amd", "csrc", "usn_device.hip")
OUT = os.path.join(ROOT, "build", "isa")
BUILDS = {"t256": (), "t512": ("USN_NTHREADS=512", "USN_NS=usn_t512")}


def _asm(name, defines):
    os.makedirs(OUT, exist_ok=True)
    return isa_check.compile_asm(SRC, os.path.join(OUT, name + ".s"), defines)


@pytest.mark.parametrize("build", sorted(BUILDS))
def test_hand_counted_waits(build):
    findings, loads = isa_check.check(_asm(build, BUILDS[build]))
    assert loads >= 20, "expected the rx hot path's asm loads, found %d" % loads
    assert not findings, "\n".join(str(f) for f in findings)


def test_check_fails_on_an_extra_load():
    text = _asm("t512_perturb1", BUILDS["t512"] + ("USN_ISA_PERTURB=1", "USN_AB_BUILD=1"))
    findings, _ = isa_check.check(text, lambda n: "classify_rx_kernelILi2ELb1" in n)
    assert any(f.kind == "loose" for f in findings), findings


def test_check_fails_on_a_stale_count():
    text = _asm("t512_perturb2", BUILDS["t512"] + ("USN_ISA_PERTURB=2", "USN_AB_BUILD=1"))
    findings, _ = isa_check.check(text, lambda n: "classify_rx_kernelILi2ELb1" in n)
    assert any(f.kind == "hazard" for f in findings), findings
