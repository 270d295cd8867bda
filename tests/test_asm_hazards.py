"""Static check (CPU, hipcc cross-compile): the inline-asm memory operations of the
cluster LSTM hand-off (csrc/lstm_coop.hip) are hazard-free in the generated gfx950 code.

* A global store of more than 8 bytes reads its data VGPRs late: the compiler pads
  the next VALU write of those registers for its own stores, but cannot see a store
  inside inline asm.  Every asm `global_store_dwordx4 ... sc1` must be followed by
  `s_nop` (>= 2 wait states) before any VALU op writes one of its data registers.
  (Round 4 found the unpadded form corrupting the backward's partial sums whenever
  the register allocator placed a v_accvgpr_read into the data registers right
  after the store.)
* An asm `global_load_dwordx4 ... sc1` is asynchronous: no instruction may read its
  destination registers before the asm `s_waitcnt vmcnt(0)` that completes it."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "information-retrieval-with-contrastive-learning_amd", "csrc")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


def _regs(tok):
    m = re.match(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    return {int(m.group(1))} if m else set()


def _instrs(lines):
    """(index, text) of real instructions (no labels, directives or asm markers)."""
    for i, l in enumerate(lines):
        t = l.strip()
        if not t or t.startswith(";") or t.startswith(".") or t.endswith(":"):
            continue
        yield i, t.split(";")[0].strip()


@pytest.fixture(scope="module")
def lstm_coop_asm(tmp_path_factory):
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    out = tmp_path_factory.mktemp("asm") / "lstm_coop.s"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17",
                    "-I" + os.path.join(ROOT, "include"), "-I" + CSRC, "--cuda-device-only",
                    "-S", os.path.join(CSRC, "lstm_coop.hip"), "-o", str(out)],
                   check=True, capture_output=True)
    return [t for _, t in _instrs(out.read_text().split("\n"))]


def test_asm_wide_stores_are_padded(lstm_coop_asm):
    ins = lstm_coop_asm
    n = 0
    for i, t in enumerate(ins):
        m = re.match(r"global_store_dwordx4 \S+, (v\[\d+:\d+\]), off sc1", t)
        if not m:
            continue
        n += 1
        data = _regs(m.group(1))
        waits = 0
        for t2 in ins[i + 1:i + 4]:
            if waits >= 2:
                break
            s = re.match(r"s_nop (\d+)", t2)
            if s:
                waits += int(s.group(1)) + 1
                continue
            d = re.match(r"v_\S+\s+(v\[\d+:\d+\]|v\d+)", t2)
            assert not (d and _regs(d.group(1)) & data), \
                f"VALU write of store data {m.group(1)} {waits} wait states after: {t} -> {t2}"
            waits += 1
    assert n > 0, "no asm wide stores found (the check would be vacuous)"


def test_asm_loads_untouched_until_waited(lstm_coop_asm):
    ins = lstm_coop_asm
    pending = set()
    n = 0
    for t in ins:
        m = re.match(r"global_load_dwordx4 (v\[\d+:\d+\]), \S+, off sc1", t)
        if m:
            pending |= _regs(m.group(1))
            n += 1
            continue
        if t.startswith("s_waitcnt") and "vmcnt(0)" in t:
            pending.clear()
            continue
        if not pending or t.startswith("s_"):
            continue
        ops = re.findall(r"v\[\d+:\d+\]|v\d+", t)
        used = set().union(*(_regs(o) for o in ops)) if ops else set()
        assert not (used & pending), f"register of an un-waited asm load touched: {t}"
    assert n > 0, "no asm loads found (the check would be vacuous)"


# gfx950 (CDNA3/4 XDL): wait states a VMEM instruction that READS a VGPR written by an
# MFMA needs after it: 16x16 shapes (8 passes) 11, 32x32 shapes (16 passes) 19.
def _mfma_wait_states(op):
    return 19 if "32x32" in op else 11


def test_asm_wide_stores_after_mfma_writes(lstm_coop_asm):
    """The backward's asm stores publish MFMA accumulators: the compiler pads an
    MFMA-write -> VMEM-read dependency for its own stores, not for one inside inline
    asm, so the instructions between the last MFMA writing a store's data registers
    and the store must cover the XDL -> VMEM-read wait states (advisor, round 4)."""
    ins = lstm_coop_asm
    n = 0
    for i, t in enumerate(ins):
        m = re.match(r"global_store_dwordx4 \S+, (v\[\d+:\d+\]), off sc1", t)
        if not m:
            continue
        n += 1
        pending = _regs(m.group(1))  # data registers whose last writer is not yet found
        waits = 0
        for t2 in reversed(ins[max(0, i - 40):i]):
            if not pending or re.match(r"s_(cbranch|branch|endpgm|setpc|swappc)", t2):
                break  # straight-line window only
            d = re.match(r"(v_mfma\S*)\s+(v\[\d+:\d+\]|v\d+)", t2)
            if d and _regs(d.group(2)) & pending:
                need = _mfma_wait_states(d.group(1))
                assert waits >= need, \
                    f"asm store of {m.group(1)} {waits} wait states after {t2} (needs {need})"
                pending -= _regs(d.group(2))
            else:
                w = re.match(r"(v_\S+)\s+(v\[\d+:\d+\]|v\d+)", t2)
                if w:  # a VALU op wrote these last: no XDL dependency for them
                    pending -= _regs(w.group(2))
            s = re.match(r"s_nop (\d+)", t2)
            waits += int(s.group(1)) + 1 if s else 1
    assert n > 0, "no asm wide stores found (the check would be vacuous)"
