"""Static ISA audit of libsvae (scripts/isa_audit.py) on CPU: hipcc compiles every kernel source to gfx950 assembly and
every inline-asm LDS-DMA statement is checked for the VALU-write-SGPR -> VMEM-read hazard on its buffer descriptor
(5 wait states; hipcc does not pad the inside of an asm statement) and for foreign m0 use; the attention backward's
q-tile loop must stay free of spill reloads, and the product GEMM instantiations (the C2 / C4 / C5 step traces) of VGPR
spills."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = '/opt/rocm/bin/hipcc'


@pytest.mark.skipif(not os.path.exists(HIPCC), reason='needs hipcc')
def test_isa_has_no_dma_hazards_and_no_spills_in_the_attention_loops(tmp_path):
    out = tmp_path / 'audit.json'
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'scripts', 'isa_audit.py'), '--quiet', '--keep',
                        str(tmp_path), '--json', str(out)], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    assert r.stdout.strip().endswith('0 hazard(s)')
    rep = json.loads(out.read_text())
    assert sum(v['dma'] for v in rep.values()) > 500          # the audit saw the DMA statements
    bwd8 = {k: v for k, v in rep.items() if 'attn_bwd8_kernel' in k}
    assert len(bwd8) == 4                                   # <hd 64 | 96, one | two 256-key sub-blocks per plane>
    for k, v in bwd8.items():
        assert v['scratch_in_mfma_loops'] == 0 and v['scratch_in_loops'] == 0, (k, v)
    # the 32x32-MFMA forward at the product occupancy (3 workgroups per CU): no spill code in its key loop
    fwd32 = {k: v for k, v in rep.items() if 'attn_fwd32_kernelILi64ELi3E' in k}
    assert len(fwd32) == 2
    for k, v in fwd32.items():
        assert v['scratch'] == 0, (k, v)

    # every gemm256 instantiation the C2 / C4 / C5 steps launch (rocprof traces): no VGPR spill (a spill reload's
    # compiler vmcnt(0) drains the DMA ring) -- <a_t, b_t, epilogue>: 0 bf16, 1 f32 (+ residual), 4 GELU, 5 GELU',
    # 6 dropout + residual, 7 rotary, 9 CE_PROB head forward, 10 head dX, 64 k-weighted head dW, 67 split-K slab (and
    # the paired slab launch); the C4 / C5 head dW in two slabs (66) keeps its few spills outside the K loop
    product = ['gemm256_kernelILb0ELb0ELi%dE' % e for e in (0, 1, 4, 5, 6, 7, 9, 10)]
    product += ['gemm256_kernelILb1ELb1ELi64E', 'gemm256_kernelILb1ELb1ELi67E', 'gemm256_pair_kernelILb1ELb1ELi67E']
    for name in product:
        hits = {k: v for k, v in rep.items() if name in k}
        assert len(hits) == 1, (name, sorted(hits))
        for k, v in hits.items():
            assert v['vgpr_spill'] == 0 and v['scratch'] == 0, (k, v)
    # the k-weighted head dW's asm dword loads (kw_pre) were checked for an early use of their destination (ASYNC_EARLY_USE)
    assert sum(v['async_loads'] for k, v in rep.items() if 'gemm256' in k and ('ELi64E' in k or 'ELi66E' in k)) >= 3
    kw2 = {k: v for k, v in rep.items() if 'gemm256_kernelILb1ELb1ELi66E' in k}
    assert len(kw2) == 1 and all(v['scratch_in_mfma_loops'] == 0 for v in kw2.values()), kw2
