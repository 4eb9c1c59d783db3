"""CPU guard of the round-4 ISA audit: the shipped code objects of the hot kernels
keep the memory-wait shape the audit fixed.  Each case disassembles one kernel symbol of the built
libskeldiff.so (llvm-objdump --disassemble-symbols) and checks its s_waitcnt / load / store order:

* k_gl4t (tiled GEMM phase, register-x fill-first ring; the N = 768 and N = 192 forms): the bias is loaded before the K loop, so the
  epilogue has no global load and no vmcnt wait between its stores; the K loop waits with counts
  (vmcnt(5) at two chunks in flight), vmcnt(0) only for the last chunk;
* k_attention<4, 32> (MANO attention): every K / Q / V load issued before the first vmcnt wait
  (one memory round trip per wave, not one per 16-node tile);
* k_gl5_mixd (MANO mixing pass): no vmcnt(0) between a row's fill and its stores;
* k_update_mfma<16, 4, 6> f32 form: no bf16 (ushort) load path.

Safety waits (round 5) -- the correctness of two hand-counted rings rests on
waits the compiler's waitcnt pass does not place by itself:

* k_gl4t's LDS-DMA ring: every s_barrier is directly preceded by an s_waitcnt that drains
  lgkmcnt(0), so no wave reaches the barrier with an LDS read of the previous chunk in flight (the
  fill issued after the barrier into that slot raced such a read in the round-4 first cut:
  test_row_chains_share_cus_bitwise[3-0] 6.6e-5 off);
* k_gl5_mixd<8, 1, true>: the residual of row r is read by inline-asm ds_read_b128 that the
  waitcnt pass cannot see; each such read group follows an s_barrier that follows the row's
  counted vmcnt wait, with no LDS-DMA issued in between, and an lgkmcnt(0) drains the reads before
  the next fill is issued.
"""
import os
import re
import shutil
import subprocess

import pytest

from conftest import REPO
from skeletondiffusion_amd import isa_check

LIB = os.path.join(REPO, "skeletondiffusion_amd", "libskeldiff.so")
OBJDUMP = shutil.which("llvm-objdump") or "/opt/rocm/lib/llvm/bin/llvm-objdump"

pytestmark = pytest.mark.skipif(not os.path.exists(OBJDUMP) or not os.path.exists(LIB), reason="no llvm-objdump / library")

GL4T = "_ZN2sd6k_gl4tILb0ELi0ELi6ELi12ELb0ELi1ELi2EEEvNS_6GLArgsEilNS_4YOutE"  # N = 768 form (CT 6, one row tile)
GL4T_RT2 = "_ZN2sd6k_gl4tILb0ELi0ELi3ELi12ELb0ELi2ELi2EEEvNS_6GLArgsEilNS_4YOutE"  # N = 192 form (CT 3, two row tiles)
ATTN = "_ZN2sd11k_attentionILi4ELi32EEEvNS_8AttnArgsE"
MIXD = "_ZN2sd12_GLOBAL__N_110k_gl5_mixdILi8ELi1ELb0EEEvNS_6GLArgsEPKfl"
MIXD_RES = "_ZN2sd12_GLOBAL__N_110k_gl5_mixdILi8ELi1ELb1EEEvNS_6GLArgsEPKfl"
UPD = "_ZN2sd13k_update_mfmaILi16ELi4ELi6ELb0EEEvNS_7UpdArgsE"

_cache = {}


def _objects(tmp_dir):
    if "objs" not in _cache:
        paths = []
        for i, (_t, b) in enumerate(isa_check.code_objects(LIB)):
            path = os.path.join(tmp_dir, f"co{i}.o")
            with open(path, "wb") as f:
                f.write(b)
            paths.append(path)
        _cache["objs"] = paths
    return _cache["objs"]


def _disasm(tmp_path_factory, sym):
    """Instruction mnemonics + operands of one kernel symbol, in program order."""
    d = str(tmp_path_factory.getbasetemp())
    for path in _objects(d):
        out = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", f"--disassemble-symbols={sym}", path],
                             capture_output=True, text=True).stdout
        lines = [l.split("//")[0].strip() for l in out.splitlines()]
        ins = [l for l in lines if l and not l.endswith(":") and not l.startswith(("Disassembly", "file format"))]
        if any(re.match(r"s_endpgm", l) for l in ins):
            return ins
    pytest.fail(f"symbol {sym} not found in the shipped library")


def _vmcnt(line):
    m = re.match(r"s_waitcnt\b.*vmcnt\((\d+)\)", line)
    return int(m.group(1)) if m else None


@pytest.mark.parametrize("sym,ntiles", [(GL4T, 6), (GL4T_RT2, 6)])
def test_gl4t_store_tail_has_no_load_waits(sym, ntiles, tmp_path_factory):
    ins = _disasm(tmp_path_factory, sym)
    last_barrier = max(i for i, l in enumerate(ins) if l.startswith("s_barrier"))
    tail = ins[last_barrier:]
    # the normal store tail: 6 tiles x 4 dwordx4 stores (the first row tile's; per row tile the
    # f16-range fallback -- exact_tile_f32, its own loads and waits, taken by out-of-range waves
    # alone -- follows that row tile's stores)
    stores = [i for i, l in enumerate(tail) if l.startswith("global_store")]
    n = 4 * ntiles if sym == GL4T else 4 * 3
    assert len(stores) >= n, len(stores)
    tail = tail[:stores[n - 1] + 1]
    assert not any(l.startswith("global_load") for l in tail), "a global load in the epilogue (bias?)"
    first_store = next(i for i, l in enumerate(tail) if l.startswith("global_store"))
    waits = [l for l in tail[first_store:] if _vmcnt(l) is not None]
    assert waits == [], waits
    # up to the last normal store (the out-of-range fallback after it waits for its own loads)
    counts = [_vmcnt(l) for l in ins[:last_barrier + len(tail)] if _vmcnt(l) is not None]
    assert counts.count(0) <= 3 and any(c > 0 for c in counts), counts


@pytest.mark.parametrize("sym,nmin", [(ATTN, 40)])
def test_attention_loads_issued_together(sym, nmin, tmp_path_factory):
    """Every load of a wave (K / Q fragments, V) issued before the first vmcnt wait: one memory
    latency per wave."""
    ins = _disasm(tmp_path_factory, sym)
    first_wait = next(i for i, l in enumerate(ins) if _vmcnt(l) is not None)
    loads = [i for i, l in enumerate(ins) if l.startswith("global_load")]
    assert len(loads) >= nmin and max(loads) < first_wait, (len(loads), max(loads), first_wait)


def test_mixd_rows_do_not_drain_fills(tmp_path_factory):
    ins = _disasm(tmp_path_factory, MIXD)
    # between a fill issued inside the row loop (after the first store) and the next store: no
    # vmcnt(0) (the prologue's one wait before the loop precedes every store)
    stores = [i for i, l in enumerate(ins) if l.startswith("buffer_store")]
    fills = [i for i, l in enumerate(ins) if l.startswith("global_load_lds")]
    in_loop_fills = [f for f in fills if f > stores[0]] if stores else []
    assert in_loop_fills, "no fill inside the row loop"
    for f in in_loop_fills:
        nxt = next((s for s in stores if s > f), None)
        if nxt is None:
            continue
        assert not any(_vmcnt(l) == 0 for l in ins[f:nxt]), ins[f:nxt]


@pytest.mark.parametrize("sym", [GL4T, GL4T_RT2])
def test_gl4t_no_scratch(sym, tmp_path_factory):
    """The whole-unrolled K loop with its register x ring stays in registers (round 6: unpinned
    range-guard reductions were sunk into the epilogue and spilled 62..270 VGPRs)."""
    ins = _disasm(tmp_path_factory, sym)
    assert not any(l.startswith("scratch_") for l in ins)


def test_update_f32_form_has_no_bf16_loads(tmp_path_factory):
    ins = _disasm(tmp_path_factory, UPD)
    assert any(l.startswith("global_load_dword") for l in ins)
    assert not any(l.startswith(("global_load_ushort", "global_load_short")) for l in ins)


@pytest.mark.parametrize("sym", [GL4T, GL4T_RT2])
def test_gl4t_ring_barriers_drain_lds_reads(sym, tmp_path_factory):
    ins = _disasm(tmp_path_factory, sym)
    bars = [i for i, l in enumerate(ins) if l.startswith("s_barrier")]
    assert len(bars) >= 4, len(bars)  # the unrolled ring steps (PF = 2) + the last chunks + the epilogue
    for i in bars:
        prev = ins[i - 1]
        assert prev.startswith("s_waitcnt") and "lgkmcnt(0)" in prev, (i, ins[i - 3:i + 1])
    ring = [i for i in bars if _vmcnt(ins[i - 1]) is not None]
    assert len(ring) >= 3, [ins[i - 1] for i in bars]  # ring waits: counted vmcnt AND lgkmcnt(0)


def test_mixd_residual_reads_follow_the_row_wait(tmp_path_factory):
    ins = _disasm(tmp_path_factory, MIXD_RES)
    groups = []  # runs of consecutive-ish ds_read_b128 (the asm residual reads of one row)
    for i, l in enumerate(ins):
        if l.startswith("ds_read_b128"):
            if groups and i - groups[-1][-1] <= 4:
                groups[-1].append(i)
            else:
                groups.append([i])
    groups = [g for g in groups if len(g) == 4]
    assert groups, "no residual read group (4 x ds_read_b128)"
    for g in groups:
        bar = max(i for i in range(g[0]) if ins[i].startswith("s_barrier"))
        assert not any(l.startswith("global_load_lds") for l in ins[bar:g[0]]), "a fill between the barrier and the reads"
        prev_issue = max((i for i in range(bar) if ins[i].startswith(("global_load_lds", "buffer_store"))), default=-1)
        assert any(_vmcnt(l) is not None for l in ins[prev_issue + 1:bar]), "no vmcnt wait before the row's barrier"
        nxt = next((i for i in range(g[-1], len(ins)) if ins[i].startswith("global_load_lds")), len(ins))
        assert any(l.startswith("s_waitcnt") and "lgkmcnt(0)" in l for l in ins[g[-1]:nxt]), \
            "the asm reads are not drained before the next fill"
