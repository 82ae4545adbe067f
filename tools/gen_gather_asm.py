#!/usr/bin/env python3
"""Generate the gather loop of kernel K1 (k_stream) for one register geometry.

    gen_gather_asm.py [--cw 16] [--batch 4] [--cap 24] [--budget 128] [--depth 1] [--tail 1] [-o path]

Why generated: the loop is a fully unrolled, software-pipelined sequence of
positions whose register names are static per position; writing it by hand
is error-prone, and the geometry is a tuning knob: columns per wave CW
(4*CW accumulator VGPRs), batch size, SGPR stream capacity CAP and the VGPR
budget per wave (512 / waves per SIMD).

Entries reach the wave as SCALARS.  A chunk's stream (stream layout v4,
csrc/tcsc_internal.h) is a 16-byte header {nb, rem, bytes to the next
header, 0} and then 8-byte entries {+-1.0f, (lds_row<<10) | 4*slot}; the
header and the first CAP entries sit in SGPRs s36 .. s39+2*CAP in memory
order: the kernel's C++ loads them with s_load right after the previous
gather (the compiler's SMEM, waited before this asm; its latency hides
behind the chunk barrier).  The loop counts down the header's nb in place,
reads rem from it, and ends by moving the pointer s[PTR:PTR+1] to the next
chunk's header, so the C++ around it does no per-chunk arithmetic.
Streams longer than CAP reload the entries in place between phases
(s_load at the header's address + the header's scratch dword, which each
reload advances by CAP entries; then lgkmcnt(0); rare at 98 % sparsity).

Per batch p (BATCH entries, slots j = BATCH*p + i of the phase):
  ISSUE(p): v_bfi the per-lane LDS address (word's row bits + lane*16) into
            the first register of the entry's X quad; ds_read_b128 into it.
  FMA(p):   s_waitcnt lgkmcnt(BATCH) (batch p+1's reads stay in flight),
            s_set_gpr_idx_on/idx word (low 8 bits = 4*slot) then two
            v_pk_fma_f32 acc[slot] += sign * x (DST and SRC2 relatively
            addressed), s_set_gpr_idx_off.
Position p does ISSUE(p) then FMA(p-DEPTH), so a batch's LDS latency hides
under the FMAs of the DEPTH batches before it (DEPTH*BATCH reads stay in
flight).  X quads cycle through DEPTH+1 register sets.

Stream lengths (--tail):
  1 (default) unpadded streams: nb = whole batches, rem = entries of
    the last, partial batch.  Position p first checks whether the whole
    batches are used up and, if so, jumps to tail p, which issues only the
    rem reads of batch p, finishes batch p-1 and FMAs the rem entries
    (generate_tail).  At 98 % sparsity a wave's chunk stream averages ~15
    entries, so padding to whole batches cost ~10 % of the gathers.
  0 the plan pads every stream to a multiple of BATCH with no-op entries
    (+1 x the -0.0 row) and the loop runs whole batches (generate).
tests/test_gather_gen.py runs the generated instruction lists through a
small interpreter for every stream length.

TCSC_ABLATION = 1..5 selects timing-only variants (wrong results):
1 no index mode, 3 no LDS read, 4 no FMA, 5 no gather.
"""
import argparse
import os
import sys


class Geo:
    def __init__(self, cw, batch, cap, budget, depth=1, touch=0, tail=1, hdr=4, pf=0):
        assert cw % 4 == 0 and cap % batch == 0 and 36 + hdr + 2 * cap <= 100
        assert hdr == 4 and (hdr + 2 * cap) % 4 == 0
        assert 1 <= depth and depth * batch <= 15, "lgkmcnt counts to 15"
        self.cw, self.batch, self.cap, self.budget, self.depth = cw, batch, cap, budget, depth
        self.touch = touch  # scalar-cache lines of the NEXT chunk's stream touched at the start
        self.pf = pf  # scalar-cache lines of THIS stream past the buffer, touched when it will reload
        self.tail = bool(tail)
        self.npos = cap // batch
        assert self.npos > depth
        nacc, self.nx = 4 * cw, 4 * batch * (depth + 1)
        self.xbase = (budget - self.nx) & ~3
        self.acc = (self.xbase - nacc) & ~1
        assert self.acc >= 12, "VGPR budget too small for this geometry"
        self.xset = {k: self.xbase + 4 * batch * k for k in range(depth + 1)}
        self.hdr = hdr  # chunk-header dwords ahead of the entries (stream layout v4)
        self.sbuf = 36  # first SGPR of the scalar buffer: [header][CAP entries]
        self.sbase = 36 + hdr
        self.slast = 36 + hdr + 2 * cap - 1
        # the chunk header in the buffer's first SGPRs: whole batches (the
        # loop's countdown), the rest, bytes to the next header, and a
        # scratch dword (0 in memory) the reloads use as their offset
        self.nb, self.rem, self.next, self.roff = (f"s{36 + i}" for i in range(4))
        self.ptr = self.slast + 1 + ((self.slast + 1) & 1)


ABL = 0
# SGN = 1: cost proxy of a 4-byte entry stream.  The +-1
# multiplier is rebuilt per entry from a sign bit with 2 SALU (s_and the
# bit, s_or 1.0's exponent) into a scratch SGPR pair instead of being loaded
# as the entry's own dword.  The proxy takes the bit from the 8-byte entry's
# sign dword, so results are unchanged and only the instruction cost moves.
# SGN = 2: the same 2 SALU a batch ahead (in ISSUE), in place over the sign
# dword, so no FMA waits on a just-written SGPR.
SGN = 0
SGN_BASE = 92  # scratch pairs s[92:93] .. s[98:99], one per batch entry


def sreg(g, j, w):
    """SGPR of entry slot j: w=0 sign, w=1 word."""
    return g.sbase + 2 * j + w


def issue(g, p, n=None):
    """Reads of batch p's first n entries (default: the whole batch)."""
    n = g.batch if n is None else n
    x = g.xset[p % (g.depth + 1)]
    out = []
    for i in range(n):
        out.append(f"v_bfi_b32 v{x + 4 * i}, %[mask], %[lane], s{sreg(g, g.batch * p + i, 1)}")
    if ABL != 3:
        for i in range(n):
            out.append(f"ds_read_b128 v[{x + 4 * i}:{x + 4 * i + 3}], v{x + 4 * i}")
    if SGN == 2:
        # the decode a batch ahead of its FMAs, in place over the entry's sign dword
        for i in range(n):
            sg = sreg(g, g.batch * p + i, 0)
            out += [f"s_and_b32 s{sg}, s{sg}, 0x80000000", f"s_or_b32 s{sg}, s{sg}, 0x3f800000"]
    return out


def fma(g, p, wait, n=None):
    """FMAs of batch p's first n entries after waiting for all but `wait` LDS reads."""
    n = g.batch if n is None else n
    x = g.xset[p % (g.depth + 1)]
    out = []
    if SGN == 1 and ABL != 4:
        for i in range(n):
            t = SGN_BASE + 2 * i
            out += [f"s_and_b32 s{t}, s{sreg(g, g.batch * p + i, 0)}, 0x80000000", f"s_or_b32 s{t}, s{t}, 0x3f800000"]
    out.append(f"s_waitcnt lgkmcnt({wait})")
    if ABL == 4:
        return out
    for i in range(n):
        j = g.batch * p + i
        w1, sg = sreg(g, j, 1), sreg(g, j, 0)
        pair = f"s[{SGN_BASE + 2 * i}:{SGN_BASE + 2 * i + 1}]" if SGN == 1 else f"s[{sg}:{sg + 1}]"
        a = g.acc + 4 * (i % g.cw) if ABL == 1 else g.acc
        if ABL != 1:
            out.append(f"s_set_gpr_idx_on s{w1}, gpr_idx(SRC2,DST)" if i == 0 else f"s_set_gpr_idx_idx s{w1}")
        out.append(f"v_pk_fma_f32 v[{a}:{a + 1}], v[{x + 4 * i}:{x + 4 * i + 1}], {pair}, v[{a}:{a + 1}] op_sel_hi:[1,0,1]")
        out.append(f"v_pk_fma_f32 v[{a + 2}:{a + 3}], v[{x + 4 * i + 2}:{x + 4 * i + 3}], {pair}, v[{a + 2}:{a + 3}] op_sel_hi:[1,0,1]")
    if ABL != 1:
        out.append("s_set_gpr_idx_off")
    return out


def count(g, p, target):
    """After ISSUE(p): was batch p the phase's last one?  (nb is the number
    of batches left in this phase and beyond; 2 SALU, no decrement.)"""
    return [f"s_cmp_eq_u32 {g.nb}, {p + 1}", f"s_cbranch_scc1 {target}"]


def reload(g):
    """Next CAP entries of this stream into the buffer (phase > 0): from the
    chunk header's address (s[PTR:PTR+1], TCSC_PTR_OPERAND, unchanged) plus
    the header's scratch dword, advanced by CAP entries per phase."""
    ptr = g.ptr
    out = [f"s_add_u32 {g.roff}, {g.roff}, {8 * g.cap}"]
    nd = 2 * g.cap
    off = 4 * g.hdr  # the pointer is the chunk header's address
    r = g.sbase
    while nd > 0:
        w = 16 if nd >= 16 and r % 4 == 0 else 8 if nd >= 8 and r % 4 == 0 else 4 if nd >= 4 and r % 4 == 0 else 2
        out.append(f"s_load_dwordx{w} s[{r}:{r + w - 1}], s[{ptr}:{ptr + 1}], {g.roff} offset:{hex(off)}")
        r += w
        off += 4 * w
        nd -= w
    out.append("s_waitcnt lgkmcnt(0)")
    return out


def advance(g):
    """Leave the pointer at the next chunk's header (the chain, stream layout v4)."""
    return [f"s_add_u32 s{g.ptr}, s{g.ptr}, {g.next}", f"s_addc_u32 s{g.ptr + 1}, s{g.ptr + 1}, 0"]


def generate(g):
    if ABL == 5:
        return []
    D = g.depth

    def drain(last):
        """FMA the batches still in flight after ISSUE(last), oldest first."""
        out = []
        for q in range(max(0, last - D + 1), last + 1):
            out += fma(g, q, g.batch * (last - q))
        return out

    L = touch(g)
    L += [f"s_cmp_eq_u32 {g.nb}, 0", "s_cbranch_scc1 .Lend%="]
    L.append(".Lphase%=:")
    for p in range(g.npos):
        L += issue(g, p)
        if p >= D:
            L += fma(g, p - D, g.batch * D)
        L += count(g, p, f".Ldrain{p}%=")
    # a full phase done with batches left: finish its batches, reload, go on
    L += drain(g.npos - 1)
    L.append(f"s_sub_u32 {g.nb}, {g.nb}, {g.npos}")
    L += reload(g)
    L.append("s_branch .Lphase%=")
    for p in range(g.npos):
        L.append(f".Ldrain{p}%=:")
        L += drain(p)
        if p != g.npos - 1:
            L.append("s_branch .Lend%=")
    L.append(".Lend%=:")
    if g.touch:
        L.append("s_waitcnt lgkmcnt(0)")  # touches still in flight must land before %[junk] is released
    return L + advance(g)


def touch(g):
    """Warm the scalar cache with the NEXT chunk's stream: its header is
    `next` bytes past this one's (the header's third dword, an SGPR offset
    of the load), so the real s_load after this gather hits K$ instead of
    paying an L2 round trip on the critical path after the barrier.  The
    loads land in the junk SGPR (pinned, never read); while one is in
    flight a counted LDS wait may wait for one more read, never fewer."""
    return [f"s_load_dword %[junk], s[{g.ptr}:{g.ptr + 1}], {g.next} offset:{hex(64 * t)}" for t in range(g.touch)]


def generate_tail(g):
    """Unpadded streams: %[nb] whole batches + %[rem] (0 .. BATCH-1) entries.
    The steady state issues exactly what the padded loop issues (the
    end-of-stream check moves ahead of ISSUE); only the last batch differs.
    Tail p: the DEPTH batches before p are issued, not yet FMA'd; it issues
    the rem reads of batch p, FMAs those batches oldest first, then the rem
    entries."""
    if ABL == 5:
        return []
    D = g.depth
    L = touch(g) + prefetch(g)
    L.append(".Lphase%=:")
    for p in range(g.npos):
        L += [f"s_cmp_eq_u32 {g.nb}, {p}", f"s_cbranch_scc1 .Ltail{p}%="]
        L += issue(g, p)
        if p >= D:
            L += fma(g, p - D, g.batch * D)
    # a full phase with batches left: finish its last batches, reload, go on
    for q in range(g.npos - D, g.npos):
        L += fma(g, q, g.batch * (g.npos - 1 - q))
    L.append(f"s_sub_u32 {g.nb}, {g.nb}, {g.npos}")
    L += reload(g)
    L.append("s_branch .Lphase%=")
    for p in range(g.npos):
        L.append(f".Ltail{p}%=:")
        for r in range(g.batch - 1):
            L += [f"s_cmp_eq_u32 {g.rem}, {r}", f"s_cbranch_scc1 .Lt{p}r{r}%="]
        for r in range(g.batch - 1, -1, -1):
            L.append(f".Lt{p}r{r}%=:")
            L += issue(g, p, r)
            for q in range(max(0, p - D), p):
                L += fma(g, q, g.batch * (p - 1 - q) + r)
            if r:
                L += fma(g, p, 0, r)
            if not (p == g.npos - 1 and r == 0):
                L.append("s_branch .Lend%=")
    L.append(".Lend%=:")
    if g.pf or g.touch:
        L.append("s_waitcnt lgkmcnt(0)")  # a touch still in flight must land before %[junk] is released
    return L + advance(g)


def prefetch(g):
    """Streams longer than the buffer reload in place with an exposed scalar
    load (cfg 2: ~38 entries per wave and chunk against 24).  When the header
    says so (nb >= whole batches of a phase), touch the scalar-cache lines the
    first reload will read, so it hits.  The touches land in %[junk]; while
    they are in flight the counted LDS waits are conservative, never wrong."""
    if not g.pf:
        return []
    first = 4 * g.hdr + 8 * g.cap  # bytes the buffer already holds
    line0 = (first + 63) // 64 * 64
    L = [f"s_cmp_lt_u32 {g.nb}, {g.npos}", "s_cbranch_scc1 .Lnopf%="]
    L += [f"s_load_dword %[junk], s[{g.ptr}:{g.ptr + 1}], {hex(line0 + 64 * i)}" for i in range(g.pf)]
    L.append(".Lnopf%=:")
    return L


def emit(f, name, lines):
    f.write(f"#define {name} \\\n")
    for l in lines:
        f.write(f'    "{l}\\n\\t" \\\n')
    f.write('    ""\n')


def write_inc(path, g):
    global ABL
    aw = 32 if (4 * g.cw) % 32 == 0 else 16  # accumulator vector width (asm operands)
    nvec = 4 * g.cw // aw
    ndw = g.hdr + 2 * g.cap      # scalar buffer: header + entries
    nsv = ndw // 16              # 16-SGPR vectors of the buffer
    stail = ndw % 16             # + one 4- or 8-SGPR vector
    assert stail in (0, 4, 8, 12)
    with open(path, "w") as f:
        f.write("// GENERATED by tools/gen_gather_asm.py -- do not edit by hand.\n")
        f.write(f"// geometry: cw={g.cw} batch={g.batch} cap={g.cap} vgpr budget={g.budget} depth={g.depth} "
                f"tail={int(g.tail)}: "
                f"acc v[{g.acc}:{g.acc + 4 * g.cw - 1}], X v[{g.xbase}:{g.xbase + g.nx - 1}], "
                f"stream s[{g.sbase}:{g.slast}]\n")
        f.write(f"#define TCSC_GEN_CW {g.cw}\n#define TCSC_GEN_BATCH {g.batch}\n#define TCSC_GEN_CAP {g.cap}\n")
        f.write(f"#define TCSC_GEN_HDR {g.hdr}\n")
        f.write(f"#define TCSC_GEN_BUDGET {g.budget}\n#define TCSC_ACC_W {aw}\n#define TCSC_ACC_VECS {nvec}\n#define TCSC_SBUF_VECS {nsv}\n")
        f.write(f"#define TCSC_SBUF_TAIL {stail}\n")
        f.write(f"#define TCSC_GEN_TAIL {int(g.tail)}\n")
        ops = ", ".join(f'"+{{v[{g.acc + aw * i}:{g.acc + aw * i + aw - 1}]}}"(acc[{i}])' for i in range(nvec))
        f.write(f"#define TCSC_ACC_OPERANDS(acc) {ops}\n")
        sops = ", ".join(f'"+{{s[{g.sbuf + 16 * i}:{g.sbuf + 16 * i + 15}]}}"(sb[{i}])' for i in range(nsv))
        if stail:
            t0 = g.sbuf + 16 * nsv
            sops += f', "+{{s[{t0}:{t0 + stail - 1}]}}"(sbt)'
        f.write(f"#define TCSC_SBUF_OPERANDS(sb, sbt) {sops}\n")
        ptr = g.ptr
        f.write(f'#define TCSC_PTR_OPERAND(p) "+{{s[{ptr}:{ptr + 1}]}}"(p)\n')
        if g.touch:
            f.write(f'#define TCSC_JUNK_OPERAND(j) [junk] "+{{s{ptr + 2}}}"(j)\n')
        else:
            f.write('#define TCSC_JUNK_OPERAND(j) [junk] "+s"(j)\n')
        f.write(f"#define TCSC_GEN_TOUCH {g.touch}\n")
        f.write(f"#define TCSC_GEN_PF {g.pf}\n")
        clob = ['"memory"', '"scc"']
        clob += [f'"v{r}"' for r in range(g.xbase, g.xbase + g.nx)]
        if SGN == 1:
            clob += [f'"s{r}"' for r in range(SGN_BASE, SGN_BASE + 2 * g.batch)]
        f.write("#define TCSC_GATHER_CLOBBERS " + ", ".join(clob) + "\n")
        f.write("#if !defined(TCSC_ABLATION) || TCSC_ABLATION == 0 || TCSC_ABLATION >= 6\n")
        for a in (0, 1, 3, 4, 5):
            if a:
                f.write(f"#elif TCSC_ABLATION == {a}\n")
            ABL = a
            body = generate_tail(g) if g.tail else generate(g)
            # s_set_gpr_idx_on/idx write M0[7:0]: the loop saves and restores
            # M0 (operand %[m0sv]), so no compiler-managed M0 value is lost
            # (M0 is a reserved register: a clobber would not be honoured)
            emit(f, "TCSC_GATHER_ASM", ["s_mov_b32 %[m0sv], m0"] + body + ["s_mov_b32 m0, %[m0sv]"] if body else [])
        f.write("#else\n#define TCSC_GATHER_ASM \"\"\n#endif\n")
        ABL = 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cw", type=int, default=16)
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--cap", type=int, default=24)
    ap.add_argument("--budget", type=int, default=128)
    ap.add_argument("--depth", type=int, default=1)
    ap.add_argument("--touch", type=int, default=0)
    ap.add_argument("--tail", type=int, default=1)
    ap.add_argument("--hdr", type=int, default=4, help="chunk-header dwords ahead of the entries")
    ap.add_argument("--pf", type=int, default=0, help="scalar-cache lines prefetched for a stream that will reload")
    ap.add_argument("--sgn", type=int, default=0, help="1/2: rebuild the +-1 multiplier from a sign bit (2 SALU per entry; 2: a batch ahead)")
    here = os.path.dirname(os.path.abspath(__file__))
    ap.add_argument("-o", default=os.path.join(here, "..", "sparse-matrix-multiplication-benchmark_amd", "csrc",
                                               "gather_asm.inc"))
    a = ap.parse_args()
    global SGN
    SGN = a.sgn
    write_inc(a.o, Geo(a.cw, a.batch, a.cap, a.budget, a.depth, a.touch, a.tail, a.hdr, a.pf))
    print(a.o)


if __name__ == "__main__":
    sys.exit(main())
