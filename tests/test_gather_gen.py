"""The generated gather loop (tools/gen_gather_asm.py), checked on the CPU.

A small interpreter walks the generated instruction list of k_stream's
gather for every stream length n (up to three SGPR buffers) and checks:
  * each of the n entries is read from LDS exactly once and FMA'd exactly
    twice (two v_pk_fma_f32 of 2 rows each); no entry at or past n is read
    (streams are unpadded: a stray gather would add a garbage row);
  * every FMA runs after an s_waitcnt lgkmcnt that covers its LDS read and
    uses the sign SGPRs and the gpr_idx word of the same entry as its data;
  * an X quad is not rewritten (v_bfi address or a new read) while a read
    into it is in flight or before both of its FMAs ran;
  * reloads of the SGPR buffer (streams longer than CAP) advance by CAP;
  * every path ends by moving the pointer to the next chunk's header once.
"""
import importlib.util
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_spec = importlib.util.spec_from_file_location("gen_gather_asm", os.path.join(ROOT, "tools", "gen_gather_asm.py"))
gen = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(gen)

RE_BFI = re.compile(r"v_bfi_b32 v(\d+), %\[mask\], %\[lane\], s(\d+)$")
RE_DS = re.compile(r"ds_read_b128 v\[(\d+):(\d+)\], v(\d+)$")
RE_WAIT = re.compile(r"s_waitcnt lgkmcnt\((\d+)\)$")
RE_IDX = re.compile(r"s_set_gpr_idx_(?:on|idx) s(\d+)")
RE_FMA = re.compile(r"v_pk_fma_f32 v\[(\d+):\d+\], v\[(\d+):\d+\], s\[(\d+):\d+\], v\[(\d+):\d+\] op_sel_hi:\[1,0,1\]$")
RE_CMP = re.compile(r"s_cmp_eq_u32 (s\d+), (\d+)$")
RE_CMPLT = re.compile(r"s_cmp_lt_u32 (s\d+), (\d+)$")
RE_SUB = re.compile(r"s_sub_u32 (s\d+), (s\d+), (\d+)$")
RE_ADD = re.compile(r"s_add_u32 (s\d+), (s\d+), (\d+)$")
RE_ADV = re.compile(r"s_add_u32 (s\d+), (s\d+), (s\d+)$")
IGNORED = ("s_addc_u32", "s_load_dword", "s_set_gpr_idx_off")


def simulate(g, lines, nb, rem):
    """Run the loop for a stream of nb whole batches + rem entries; returns
    (reads, fmas): how often each entry index was read / FMA'd."""
    labels = {ln[:-1]: i for i, ln in enumerate(lines) if ln.endswith(":")}
    ptr = f"s{g.ptr}"
    n = nb * g.batch + rem
    regs = {g.nb: nb, g.rem: rem}
    advanced = 0
    base = 0  # stream index of SGPR slot 0
    scc = False
    addr, quad, pending = {}, {}, []  # address VGPR -> entry; quad -> [entry, landed, fmas]; reads in flight
    idx_entry = None
    reads, fmas = {}, {}

    def entry(sreg, word):
        j, r = divmod(sreg - g.sbase - word, 2)
        assert r == 0 and 0 <= j < g.cap, f"s{sreg} is not a stream slot"
        return base + j

    def quad_of(v):
        assert g.xbase <= v < g.xbase + g.nx, f"v{v} is not an X register"
        return g.xbase + (v - g.xbase) // 4 * 4

    pc = steps = 0
    while pc < len(lines):
        steps += 1
        assert steps < 100000, "no exit"
        ln = lines[pc]
        pc += 1
        if ln.endswith(":") or ln.startswith(IGNORED):
            continue
        if m := RE_CMP.match(ln):
            scc = regs[m[1]] == int(m[2])
        elif m := RE_CMPLT.match(ln):
            scc = regs[m[1]] < int(m[2])
        elif ln.startswith("s_cbranch_scc1 "):
            if scc:
                pc = labels[ln.split()[1]]
        elif ln.startswith("s_branch "):
            pc = labels[ln.split()[1]]
        elif m := RE_BFI.match(ln):
            v = int(m[1])
            assert v == quad_of(v) and v not in pending, f"v{v}: address written while a read into it is in flight"
            assert v not in quad or quad[v][2] == 2, f"quad v{v} reused before its FMAs"
            addr[v] = entry(int(m[2]), 1)
        elif m := RE_DS.match(ln):
            q = int(m[1])
            assert int(m[3]) == q == quad_of(q) and int(m[2]) == q + 3
            e = addr.pop(q)
            assert e < n, f"read of entry {e} past the stream end ({n})"
            reads[e] = reads.get(e, 0) + 1
            quad[q] = [e, False, 0]
            pending.append(q)
        elif m := RE_WAIT.match(ln):
            while len(pending) > int(m[1]):
                quad[pending.pop(0)][1] = True
        elif m := RE_IDX.match(ln):
            idx_entry = entry(int(m[1]), 1)
        elif m := RE_FMA.match(ln):
            acc, x, s, acc2 = (int(m[i]) for i in (1, 2, 3, 4))
            q = quad_of(x)
            assert acc == acc2 and acc - g.acc == x - q in (0, 2), "row pair of quad and accumulator differ"
            e, landed, done = quad[q]
            assert landed, f"FMA of entry {e} before its read is waited for"
            assert entry(s, 0) == e == idx_entry, "sign / index / data of different entries"
            quad[q][2] = done + 1
            fmas[e] = fmas.get(e, 0) + 1
        elif m := RE_SUB.match(ln):
            assert m[1] == m[2] == g.nb
            regs[g.nb] -= int(m[3])
        elif m := RE_ADD.match(ln):
            assert m[1] == m[2] == g.roff and int(m[3]) == 8 * g.cap, ln
            base += g.cap
        elif m := RE_ADV.match(ln):
            assert m[1] == m[2] == ptr and m[3] == g.next, ln
            advanced += 1
        else:
            raise AssertionError(f"unexpected instruction {ln!r}")
    assert advanced == 1, "the pointer must end at the next chunk's header, once"
    return reads, fmas


GEOS = [dict(cw=16, batch=4, cap=24), dict(cw=16, batch=4, cap=16), dict(cw=16, batch=6, cap=24),
        dict(cw=16, batch=2, cap=24)]


@pytest.mark.parametrize("touch", [0, 2])
@pytest.mark.parametrize("pf", [0, 3])
@pytest.mark.parametrize("depth", [1, 2])
@pytest.mark.parametrize("geo", GEOS, ids=lambda d: "b{batch}_c{cap}".format(**d))
def test_tail_loop_gathers_each_entry_once(geo, depth, pf, touch):
    try:
        g = gen.Geo(budget=128, depth=depth, touch=touch, tail=1, pf=pf, **geo)
    except AssertionError as e:
        pytest.skip(f"geometry not valid at this depth: {e}")
    lines = gen.generate_tail(g)
    if touch or pf:  # the junk SGPR's loads have landed before the loop hands it back
        assert lines[lines.index(".Lend%=:") + 1] == "s_waitcnt lgkmcnt(0)"
    for n in range(3 * g.cap + 2 * g.batch + 1):
        reads, fmas = simulate(g, lines, n // g.batch, n % g.batch)
        assert sorted(reads) == list(range(n)) and set(reads.values()) <= {1}, n
        assert sorted(fmas) == list(range(n)) and set(fmas.values()) <= {2}, n


@pytest.mark.parametrize("depth", [1, 2])
def test_padded_loop_gathers_whole_batches(depth):
    g = gen.Geo(16, 4, 24, 128, depth=depth, touch=0, tail=0)
    lines = gen.generate(g)
    for nb in range(3 * g.npos + 2):
        reads, fmas = simulate(g, lines, nb, 0)
        assert sorted(reads) == list(range(nb * g.batch)) and set(reads.values()) <= {1}, nb
        assert sorted(fmas) == list(range(nb * g.batch)) and set(fmas.values()) <= {2}, nb


def test_shipped_include_matches_generator(tmp_path):
    """csrc/gather_asm.inc is what the generator writes for its defaults."""
    out = tmp_path / "gather_asm.inc"
    gen.write_inc(str(out), gen.Geo(16, 4, 24, 128, depth=1, touch=0, tail=1))
    with open(os.path.join(ROOT, "sparse-matrix-multiplication-benchmark_amd", "csrc", "gather_asm.inc")) as f:
        assert f.read() == out.read_text()
