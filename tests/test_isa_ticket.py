"""ISA-level pin of the fence-free last-block ticket (csrc/kernels/misc.hip take_ticket,
VERDICT r5 ask 6): disassemble the BUILT gfx950 code object of ``_kernels`` with ROCm's
llvm-objdump and check, for both kernels that use the protocol (``splitk_fused4_k``, the
split-K reduce; ``fused_opt_k``, the optimizer + finalize):

* the partials are stored write-through: ``global_store_* ... sc1`` before the ticket;
* the ticket is a returning agent-scope ``global_atomic_add`` preceded by an
  ``s_waitcnt vmcnt(0)`` with no vector-memory instruction in between;
* the winner reads the partials with ``global_load_* ... sc1`` after the ticket (in the
  split-K reduce: every load after the ticket).

A compiler or flag change that drops ``sc1`` (st_coh / ld_coh replaced by plain accesses) or
the wait fails here deterministically, instead of as rare wrong sums on the GPU.  CPU only.
"""
import os
import re
import struct
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
BUNDLE = b"__CLANG_OFFLOAD_BUNDLE__"
VMEM = re.compile(r"^\s*(global|buffer|flat|scratch)_")


def _code_objects(so_path):
    """gfx950 ELF code objects of every (uncompressed) clang offload bundle in the .so."""
    d = open(so_path, "rb").read()
    i = 0
    while True:
        i = d.find(BUNDLE, i)
        if i < 0:
            return
        n = struct.unpack_from("<Q", d, i + 24)[0]
        p = i + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", d, p)
            p += 24
            triple = d[p:p + tl].decode(errors="replace")
            p += tl
            if "gfx950" in triple:
                yield d[i + off:i + off + size]
        i += len(BUNDLE)


@pytest.fixture(scope="module")
def disasm():
    if not os.path.exists(OBJDUMP):
        pytest.skip("ROCm llvm-objdump not installed")
    from distributed_tensorflow_ibm_mnist_amd import _build
    so = _build.kernels_so()
    if not os.path.exists(so):
        _build.build_all(force=False, verbose=False)
    funcs = {}
    with tempfile.TemporaryDirectory() as td:
        for k, co in enumerate(_code_objects(so)):
            f = os.path.join(td, f"co{k}.elf")
            open(f, "wb").write(co)
            txt = subprocess.run([OBJDUMP, "-d", "--no-show-raw-insn", f], capture_output=True, text=True,
                                 check=True).stdout
            name, body = None, []
            for line in txt.splitlines():
                m = re.match(r"^[0-9a-f]+ <(\S+)>:$", line)
                if m:
                    if name:
                        funcs[name] = body
                    name, body = m.group(1), []
                elif name and line.startswith("\t"):
                    body.append(line.split("//")[0].strip())
            if name:
                funcs[name] = body
    assert funcs, "no gfx950 code object found in " + so
    return funcs


def _kernel(funcs, sub):
    names = [n for n in funcs if sub in n]
    assert len(names) == 1, (sub, names)
    return funcs[names[0]]


def _tickets(body):
    return [i for i, ins in enumerate(body) if ins.startswith("global_atomic_add") and " sc0" in ins]


@pytest.mark.parametrize("kernel", ["splitk_fused4_k", "fused_optk"])
def test_ticket_waits_for_coherent_stores(disasm, kernel):
    body = _kernel(disasm, "15splitk_fused4_k" if kernel == "splitk_fused4_k" else "11fused_opt_k")
    tk = _tickets(body)
    assert len(tk) == 1, f"{kernel}: expected one returning ticket atomic, found {len(tk)}"
    t = tk[0]
    # back from the atomic to the previous vector-memory instruction: a vmcnt(0) wait on the way
    waited = False
    for ins in reversed(body[:t]):
        if ins.startswith("s_waitcnt") and "vmcnt(0)" in ins:
            waited = True
            break
        assert not VMEM.match(ins), f"{kernel}: vector-memory op {ins!r} between the last wait and the ticket"
    assert waited, f"{kernel}: no s_waitcnt vmcnt(0) before the ticket atomic"
    stores = [ins for ins in body[:t] if ins.startswith("global_store")]
    assert any(ins.endswith(" sc1") or " sc1 " in ins for ins in stores), \
        f"{kernel}: no write-through (sc1) partial store before the ticket: {stores[-6:]}"
    loads = [ins for ins in body[t + 1:] if ins.startswith(("global_load", "buffer_load"))]
    coh = [ins for ins in loads if ins.endswith(" sc1") or " sc1 " in ins]
    assert coh, f"{kernel}: the winner reads no partial with an sc1 load"
    if kernel == "splitk_fused4_k":   # every partial the winner reads comes from this launch
        assert len(coh) == len(loads), f"{kernel}: plain loads after the ticket: {set(loads) - set(coh)}"
    else:                             # the l2 partial sweep: 16 sc1 loads in flight per round
        assert len(coh) >= 16, f"{kernel}: only {len(coh)} sc1 loads after the ticket"


def test_partial_stores_all_write_through(disasm):
    """splitk_fused4_k's fused-path partials: the last stores before the ticket (the four
    floats of the block's quad) are all sc1."""
    body = _kernel(disasm, "15splitk_fused4_k")
    t = _tickets(body)[0]
    stores = [ins for ins in body[:t] if ins.startswith("global_store")]
    assert len(stores) >= 4 and all(" sc1" in ins for ins in stores[-4:]), stores[-4:]
