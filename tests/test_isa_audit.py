"""Static ISA audit of libsvae (scripts/isa_audit.py) on CPU: hipcc compiles every kernel source to gfx950 assembly and
every inline-asm LDS-DMA statement is checked for the VALU-write-SGPR -> VMEM-read hazard on its buffer descriptor
(5 wait states; hipcc does not pad the inside of an asm statement) and for foreign m0 use; the attention backward's
q-tile loop must stay free of spill reloads."""
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
    assert len(bwd8) == 2
    for k, v in bwd8.items():
        assert v['scratch_in_mfma_loops'] == 0, (k, v)
    # the 32x32-MFMA forward at the product occupancy (3 workgroups per CU): no spill code in its key loop
    fwd32 = {k: v for k, v in rep.items() if 'attn_fwd32_kernelILi64ELi3E' in k}
    assert len(fwd32) == 2
    for k, v in fwd32.items():
        assert v['scratch'] == 0, (k, v)
