"""Static audit of the device ISA hipcc emits for libsvae's kernels (gfx950).

    python scripts/isa_audit.py [--keep DIR] [files...]    # default: every csrc/*.hip

What hipcc does not do for an inline-asm statement (cdna_hip_programming.md §5.7): it neither models the
instructions inside nor pads their hazards. Every LDS-DMA of this library is such a statement
(`dma16_lds` / `dma4_lds` / `dma1_lds`, common.h): `s_mov_b32 m0` + `buffer_load_* ... offen lds` reading a
buffer descriptor (and soffset) from SGPRs. A VALU instruction that writes one of those SGPRs (v_readfirstlane,
v_readlane, a VALU carry-out / compare destination) needs 5 wait states before the VMEM instruction reads it; the
hazard recognizer pads its own instructions, not ours, so a descriptor refreshed by a `readfirstlane` right in
front of the statement would be read stale (wrong source address, silently wrong LDS data).

Checks, per kernel:
  * DMA_SGPR_HAZARD  a VALU write of a descriptor / soffset SGPR of an LDS-DMA within 5 wait states before it;
  * M0_HAZARD        an LDS-DMA whose m0 write is not followed by >= 1 wait state;
  * M0_FOREIGN       a compiler instruction outside our asm that touches m0 in a kernel that also issues our DMA
                     (our statements save and restore m0, so this is informational: it should stay empty);
  * ASYNC_EARLY_USE  a register-destination load issued inside our asm (the k-weighted GEMM's one dword per lane,
                     gemm.hip `kw_pre`; the attention backward's in-kernel delta O / o_lo rows; the compiler takes the
                     value as ready when the statement ends) whose destination VGPR is read, copied or overwritten
                     before the first `s_waitcnt vmcnt(N)` that retires it (at most N vector-memory instructions issued
                     after it, in program order): a v_mov of a live-range split placed there would copy a value that has
                     not landed (silently wrong results);
  * spills           .vgpr_spill_count / .sgpr_spill_count from the kernel metadata, and how many scratch
                     instructions sit in each kernel, and how many of those sit inside a loop (a spill reload's
                     compiler vmcnt(0) inside a K-tile / q-tile loop drains the hand-counted DMA ring).
Exit status 1 if any hazard is found. Writes nothing to the source tree.
"""
import argparse
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, 'sparse-vae_amd')
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
FLAGS = ['-O3', '-std=c++17', '-fPIC', '--offload-arch=gfx950', '-munsafe-fp-atomics', '--cuda-device-only', '-S']
NO_NANS = ('attention.hip', 'gemm.hip')          # the Makefile's -fno-honor-nans files

VALU_SGPR_DST0 = re.compile(r'^v_(readfirstlane|readlane|cmpx?_\w+_e64)')
VALU_SGPR_DST1 = re.compile(r'^v_(add_co|sub_co|subrev_co|addc_co|subb_co|subbrev_co|mad_u64_u32|mad_i64_i32|'
                            r'div_scale)')
SREG = re.compile(r'^s\[?(\d+)(?::(\d+))?\]?$')


def sregs(tok):
    tok = tok.strip()
    if tok in ('vcc', 'vcc_lo', 'vcc_hi', 'exec', 'm0'):
        return {tok}
    m = re.match(r'^s\[(\d+):(\d+)\]$', tok) or re.match(r'^s(\d+)$', tok)
    if not m:
        return set()
    lo = int(m.group(1))
    hi = int(m.group(2)) if m.lastindex and m.lastindex >= 2 and m.group(2) else lo
    return {f's{i}' for i in range(lo, hi + 1)}


def wait_states(ins):
    m = re.match(r'^s_nop\s+(\d+)', ins)
    return int(m.group(1)) + 1 if m else 1


def parse(path):
    """Yields (kernel, lines) with lines = [(kind, text)], kind in {'ins', 'label', 'asm_start', 'asm_end'}."""
    kern, body = None, []
    with open(path) as f:
        lines = f.read().splitlines()
    for raw in lines:
        s = raw.strip()
        m = re.match(r'^([A-Za-z_.$][\w.$]*):', s)
        if m and not s.startswith('.L') and not s.startswith('$') and ('kernel' in m.group(1) or
                                                                           m.group(1).startswith('_Z')):
            if kern:
                yield kern, body
            kern, body = m.group(1), []
            continue
        if kern is None:
            continue
        if s.startswith('.Lfunc_end') or s.startswith('.size'):
            yield kern, body
            kern, body = None, []
            continue
        if s == ';;#ASMSTART':
            body.append(('asm_start', s))
        elif s == ';;#ASMEND':
            body.append(('asm_end', s))
        elif re.match(r'^\.?L\w+:|^; %bb', s) or re.match(r'^\.LBB\w+:', s):
            body.append(('label', s))
        elif s and not s.startswith(';') and not s.startswith('.') and not s.startswith('//'):
            body.append(('ins', s.split(';')[0].strip()))
    if kern:
        yield kern, body


def spill_meta(path):
    """{kernel symbol: (vgpr_spill, sgpr_spill, vgpr_count)} from the amdhsa metadata."""
    out = {}
    text = open(path).read()
    # metadata blocks: one per kernel, keys alphabetical; split on '  - .agpr_count'
    for blk in re.split(r'\n  - ', text.split('amdhsa.kernels:')[-1]):
        name = re.search(r'\.name:\s+(\S+)', blk)
        if not name:
            continue
        g = lambda k: int(re.search(rf'\.{k}:\s+(\d+)', blk).group(1)) if re.search(rf'\.{k}:\s+(\d+)', blk) else -1
        out[name.group(1)] = (g('vgpr_spill_count'), g('sgpr_spill_count'), g('vgpr_count'))
    return out


def loop_scratch(body):
    """Scratch (spill) instructions inside a loop (between a label and a later branch back to it), and how many of
    those sit in an innermost loop that issues MFMAs (the K-tile / q-tile loops, where a reload's vmcnt(0) drains the
    DMA ring)."""
    labels = {}
    for i, (kind, text) in enumerate(body):
        if kind == 'label':
            labels[text.split(':')[0].strip()] = i
    ranges = []
    for i, (kind, text) in enumerate(body):
        m = re.match(r'^s_c?branch\w*\s+(\.LBB\w+)', text) if kind == 'ins' else None
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            ranges.append((labels[m.group(1)], i))
    mfma = [i for i, (kind, text) in enumerate(body) if kind == 'ins' and text.startswith('v_mfma')]
    inloop = inner = 0
    for i, (kind, text) in enumerate(body):
        if kind != 'ins' or not text.startswith('scratch_'):
            continue
        enc = [(a, b) for a, b in ranges if a <= i <= b]
        if not enc:
            continue
        inloop += 1
        a, b = min(enc, key=lambda r: r[1] - r[0])      # the innermost loop holding this spill
        # ... with MFMAs on both sides of the spill inside that loop: the spill sits in the MFMA stream of a K-tile /
        # q-tile loop (an epilogue spill of a persistent tile loop has the loop's MFMAs only before it)
        inner += any(a <= j < i for j in mfma) and any(i < j <= b for j in mfma)
    return inloop, inner


VREG = re.compile(r'\bv\[(\d+):(\d+)\]|\bv(\d+)\b')


def vregs(text):
    out = set()
    for m in VREG.finditer(text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


VMEM = re.compile(r'^(buffer|global|scratch|flat)_(load|store|atomic)')


def async_early_use(body, i, dst, labels=None):
    """First instruction after the asm load at body[i] (in program order) that touches VGPR dst before a
    `s_waitcnt vmcnt(N <= 8)`, or None. The product's one such load (gemm.hip `kw_pre`) is retired by the
    vmcnt(8) that leaves exactly the K-tile's 8 DMA pieces in flight; a linear scan is the check that matters there
    (a live-range-split copy of the register would sit between the statement and that wait)."""
    for j in range(i + 1, len(body)):
        kind, text = body[j]
        if kind != 'ins':
            continue
        m = re.match(r'^s_waitcnt\b.*vmcnt\((\d+)\)', text)
        if m and int(m.group(1)) <= 8:
            return None
        if dst in vregs(text):
            return j, text
    return None


def audit_kernel(name, body):
    issues = []
    in_asm = False
    labels = {t.split(':')[0].strip(): k for k, (kind, t) in enumerate(body) if kind == 'label'}
    kernel_has_dma = any(k == 'ins' and re.search(r'offen lds$|\blds$', t) for k, t in body)
    scratch = 0
    for i, (kind, text) in enumerate(body):
        if kind == 'asm_start':
            in_asm = True
            continue
        if kind == 'asm_end':
            in_asm = False
            continue
        if kind != 'ins':
            continue
        op = text.split()[0]
        if op.startswith('scratch_') or re.search(r'buffer_(store|load)\S*.*\boff(set)?\b.*s\[0:3\]', text):
            scratch += 1
        if not in_asm and kernel_has_dma and re.search(r'(^|[\s,])m0([\s,]|$)', text):
            issues.append(('M0_FOREIGN', i, text))
        if in_asm and re.match(r'^buffer_load_dword(x[234])?$', op) and not text.rstrip().endswith('lds'):
            dst = vregs(text.split(',')[0])
            for r in dst:
                hit = async_early_use(body, i, r, labels)
                if hit:
                    issues.append(('ASYNC_EARLY_USE', i, f'{text!r}: v{r} touched by {hit[1]!r} before its wait'))
        if re.match(r'^buffer_load_\w+', op) and text.rstrip().endswith('lds'):
            ops = [o.strip() for o in text[len(op):].split(',')]
            srsrc = sregs(ops[1]) if len(ops) > 1 else set()
            soff = sregs(ops[2].split()[0]) if len(ops) > 2 else set()
            need = srsrc | soff
            # walk back over 5 wait states
            states, j, m0_gap = 0, i - 1, None
            while j >= 0 and states < 5:
                k2, t2 = body[j]
                if k2 == 'ins':
                    o2 = t2.split()[0]
                    args = [a.strip() for a in t2[len(o2):].split(',')]
                    if m0_gap is None and o2 == 's_mov_b32' and args and args[0] == 'm0':
                        m0_gap = states
                    dst = set()
                    if VALU_SGPR_DST0.match(o2) and args:
                        dst = sregs(args[0])
                    elif VALU_SGPR_DST1.match(o2) and len(args) > 1:
                        dst = sregs(args[1])
                    if dst & need:
                        issues.append(('DMA_SGPR_HAZARD', i, f'{t2!r} {states} wait states before {text!r}'))
                    states += wait_states(t2)
                j -= 1
            if m0_gap is not None and m0_gap < 1:
                issues.append(('M0_HAZARD', i, text))
    return issues, scratch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('files', nargs='*')
    ap.add_argument('--keep', default=None, help='directory for the .s files (default: a temp dir)')
    ap.add_argument('--quiet', action='store_true')
    ap.add_argument('--json', default=None, help='write the per-kernel report here')
    args = ap.parse_args()
    files = args.files or sorted(os.path.join(PKG, 'csrc', f) for f in os.listdir(os.path.join(PKG, 'csrc'))
                                 if f.endswith('.hip'))
    out_dir = args.keep or tempfile.mkdtemp(prefix='svae_isa_')
    os.makedirs(out_dir, exist_ok=True)
    procs = []
    for f in files:
        s = os.path.join(out_dir, os.path.basename(f).replace('.hip', '.s'))
        extra = ['-fno-honor-nans'] if os.path.basename(f) in NO_NANS else []
        procs.append((f, s, subprocess.Popen([HIPCC] + FLAGS + extra + [f, '-o', s], stderr=subprocess.DEVNULL)))
    bad = 0
    report = {}
    for f, s, p in procs:
        if p.wait() != 0:
            print(f'{f}: compile failed', file=sys.stderr)
            bad += 1
            continue
        meta = spill_meta(s)
        for name, body in parse(s):
            issues, scratch = audit_kernel(name, body)
            vsp, ssp, vg = meta.get(name, (-1, -1, -1))
            ndma = sum(1 for k, t in body if k == 'ins' and t.endswith(' lds'))
            nasync = sum(1 for k, t in body if k == 'ins' and re.match(r'buffer_load_dword(x[234])?$', t.split()[0]) and
                         not t.endswith('lds') and re.search(r'\boffen( offset:\d+)?$', t))
            if issues:
                bad += len(issues)
            inloop, inner = loop_scratch(body)
            report[name] = dict(dma=ndma, async_loads=nasync, vgpr=vg, vgpr_spill=vsp, sgpr_spill=ssp, scratch=scratch,
                                scratch_in_loops=inloop, scratch_in_mfma_loops=inner, hazards=len(issues))
            if issues or not args.quiet and (ndma or vsp > 0 or ssp > 0):
                print(f'{os.path.basename(f)} {name}: {ndma} LDS-DMA, vgpr {vg}, spills v{vsp}/s{ssp}, '
                      f'{scratch} scratch instructions ({inloop} inside loops, {inner} in an MFMA loop)')
            for kind, i, text in issues:
                print(f'    {kind} @{i}: {text}')
    print(f'{bad} hazard(s)')
    if args.json:
        import json
        with open(args.json, 'w') as fh:
            json.dump(report, fh, indent=1)
    return 1 if bad else 0


if __name__ == '__main__':
    sys.exit(main())
