"""Build profiles/pmc_head_gemm_c2.json from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) over the vocabulary
head GEMM (MI355X_MICROARCH.md HBM section: FETCH_SIZE x2 on gfx950 for 16-B/lane streaming reads, WRITE_SIZE exact).

    python scripts/pmc_head_json.py gpurun_out/<tag>/pmc_fetch gpurun_out/<tag>/pmc_write KERNEL_SUBSTR [CONFIG] \
        > profiles/pmc_head_gemm_<CONFIG>.json          (CONFIG: c2 (default), c4, c5 -- bench.py's per-rank shapes)
"""
import csv
import glob
import json
import sys


def values(root, counter, sub):
    path = glob.glob(f'{root}/**/*counter_collection.csv', recursive=True)[0]
    out = []
    for r in csv.DictReader(open(path)):
        if r.get('Counter_Name') == counter and sub in r['Kernel_Name']:
            out.append(float(r['Counter_Value']))
    return out


def main():
    fdir, wdir, sub = sys.argv[1], sys.argv[2], sys.argv[3]
    cfg = sys.argv[4] if len(sys.argv) > 4 else 'c2'
    f, w = values(fdir, 'FETCH_SIZE', sub), values(wdir, 'WRITE_SIZE', sub)
    V = 32768
    T, d = {'c2': (64 * 512, 512), 'c4': (64 * 1024, 768), 'c5': (32 * 2048, 768)}[cfg]
    fb = sum(f) / len(f) * 1024 * 2
    wb = sum(w) / len(w) * 1024
    rec = {
        'kernel': f'gemm256_kernel<false, false, {sub.split(",")[-1].strip(" >")}> (vocab head)',
        'config': f'{cfg} (T={T} rows, V={V}, d={d})',
        'launches_sampled': min(len(f), len(w)),
        'source': 'rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes, --kernel-include-regex on the head '
                  f'GEMM, python3 bench.py --config {cfg} --steps 10 --warmup 3 (scripts/gpu_round.sh stage m)',
        'fetch_size_kib_raw': round(sum(f) / len(f), 1),
        'write_size_kib_raw': round(sum(w) / len(w), 1),
        'corrections': 'KiB -> bytes (x1024); FETCH_SIZE x2 (gfx950 tallies 128-B requests at 64 B for 16-B/lane '
                       'streaming reads, MI355X_MICROARCH.md); WRITE_SIZE exact for 16-B/lane stores',
        'fetch_bytes_per_launch': fb,
        'write_bytes_per_launch': wb,
        'hbm_bytes_per_launch': fb + wb,
        'algorithmic_read_bytes': 2 * (T + V) * d + 4 * V + 8 * T,
        'algorithmic_write_bytes': 2 * T * V + 4 * T * (V // 128),
    }
    print(json.dumps(rec, indent=1))


if __name__ == '__main__':
    main()
