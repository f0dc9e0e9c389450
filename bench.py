"""Training-throughput benchmark of the MI355X TransformerVAE step (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c4|c5|tiny]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

`--gpus N` (N > 1) without WORLD_SIZE in the environment: this process launches the N ranks itself (one child
per GPU with the torchrun environment, as Lightning's Trainer(gpus=N) does for the reference, train.py:63-64, 94),
never touching the GPU; it exits non-zero at once when fewer than N GPUs are visible. At N > 1 the line also
carries `scaling_efficiency` against a same-run N=1 rate (all-reduce off, after the timed region) and
`exposed_comm_ms`: the part of the gradient all-reduce the backward did not hide, per step, max over ranks.

A step = TransformerVAE.training_step (forward) + loss.backward() (engine backward with the bucketed RCCL
gradient all-reduce overlapped) + on_after_backward (grad norm, KL anneal) + RAdam.step (fused clip +
update) + LambdaLR.step, on a synthetic batch resident in HBM. Weak scaling: every rank runs the per-GPU
batch of the config; value = all ranks' tokens / max-over-ranks wall time.

Rank 0 prints ONE JSON line. At N=1 it also carries:
  roofline     — the dominant kernel (the tied vocab-head GEMM, 2*T*d*V flops per launch) timed with HIP
                 events on its own stream over the timed steps, against the dense bf16 MFMA peak;
  cpu_baseline — the CPU fp32 oracle (oracle/, pinned to the reference by tests/golden) timed on this
                 host's cores on a bounded sample of the same workload;
  parity       — GPU step vs CPU oracle loss / ELBO on the C2 model at batch 2 (same weights, noise).
"""
import argparse
import json
import math
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, 'sparse-vae_amd'))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = 'training tokens/sec + ELBO match vs CPU ref, 512-tok seq, 1/2/4/8 MI355X'
CONFIGS = {
    'tiny': dict(layers=4, d=128, heads=8, L=128, B=64),
    'c2': dict(layers=6, d=512, heads=8, L=512, B=64),
    'c4': dict(layers=12, d=768, heads=8, L=1024, B=64),
    'c5': dict(layers=12, d=768, heads=8, L=2048, B=32),
    # the C2 model with the reference's default decoder attention (sparse_self_attention, attn_window_size 4)
    'c2s': dict(layers=6, d=512, heads=8, L=512, B=64, window=4),
    # the same model and tokens per batch at the sparse presets' sequence lengths (hparam_presets.py:122-171): 2 x 16384
    'c2s16k': dict(layers=6, d=512, heads=8, L=16384, B=2, window=4),
    # the pg19 preset's shape (hparam_presets.py:150-171: one 102,400-token sample per batch, attn_window_size 6)
    'c2s100k': dict(layers=6, d=512, heads=8, L=102400, B=1, window=6),
}
V, NLAT = 32768, 64
PEAK_BF16_TFLOPS = 2500.0      # MI355X dense bf16 MFMA (MI355X_MICROARCH.md, chip-level parameters)


def _dec_keys(L, window):
    """Keys per decoder query the count prices: all L (dense), or the sliding window's band -- window 32-key blocks
    plus the [CLS] block (sparse_attention.py:39-60) -- which the window kernels visit."""
    return L if not window else min(L, 32 * (window + 1))


def flops_per_token(nl, d, L, V=V, N=NLAT, window=0):
    """F_train = 3 * F_fwd (dense count, verified against torch.utils.flop_counter); window mode
    prices the decoder's scores and P.V over the band's keys instead of all L."""
    f_enc = (4 * d * d + 4 * N * d + 18 * d * d * N / L) \
        + (nl // 2 - 2) * (4 * d * d + 4 * N * d + (28 * d * d * N + 4 * N * N * d) / L) \
        + (4 * d * d * N + 4 * N * d + 18 * d * d) / L
    f_fwd = nl * (24 * d * d + 4 * _dec_keys(L, window) * d) + 2 * d * d + 2 * d * V + f_enc
    return 3 * f_fwd


def flops_per_token_causal(nl, d, L, V=V, N=NLAT, window=0):
    """The causal-useful count: the dense count less the masked decoder attention: the upper half
    (nl * 2 * L * d per token forward), or in window mode everything past the keys a query actually sees (on average
    window - 1 full blocks, half its own block and the [CLS] block: 32 (window - 1) + 48)."""
    useful = L / 2 if not window else min(L / 2, 32 * (window - 1) + 48)
    return flops_per_token(nl, d, L, V, N, window) - 3 * nl * 4 * (_dec_keys(L, window) - useful) * d


def build(cfg, device):
    from sparse_vae import TransformerVAE, TransformerVAEHparams, TextDataModule
    hp = TransformerVAEHparams(d_model=cfg['d'], num_layers=cfg['layers'], num_heads=cfg['heads'], latent_depth=64,
                               sparse_self_attention=bool(cfg.get('window')), attn_window_size=cfg.get('window', 4),
                               grad_clip_threshold=150.0, init_scale=0.02,
                               kl_weight_start=0.3, kl_weight_end=1.0, kl_annealing_steps=8000, lr=3e-4)
    model = TransformerVAE(hp, device=device)
    model.initialize_weights()
    model.on_train_start()
    dm = TextDataModule(dataset_name='synthetic', seq_len=cfg['L'], batch_size=cfg['B'],
                        seed=7295 + 17 * int(os.environ.get('RANK', '0')))
    batch = dm.synthetic_batch(0, device=device)                  # resident in HBM before timing
    [opt], [sch] = model.configure_optimizers(cfg['B'] * cfg['L'], 1)
    return model, opt, sch['scheduler'], batch


def step(model, opt, sched, batch):
    out = model.training_step(batch, 0)
    out['loss'].backward()
    model.on_after_backward()
    opt.step()
    sched.step()
    opt.zero_grad()
    return out


def host_cores():
    """CPUs this process may use: the affinity mask, capped by the cgroup CPU quota when one is set (a GPU box
    shares its host; the quota, not the machine's CPU count, is what the process gets)."""
    n = len(os.sched_getaffinity(0))
    try:
        with open('/sys/fs/cgroup/cpu.max') as f:
            quota, period = f.read().split()[:2]
        if quota != 'max':
            n = min(n, max(1, int(int(quota) / int(period))))
    except (OSError, ValueError):
        pass
    return n


def cpu_baseline(cfg):
    """The oracle's fp32 fwd+bwd on the host cores on the config's own batch: one warm-up step at
    batch 2 (thread pool, allocator), then ONE timed step at the full per-GPU batch (C2: 64 x 512 tokens, ~10-30
    s on 8-16 cores)."""
    if cfg['L'] > 4096:
        # (the oracle's attention is dense: at 16 K tokens its autograd keeps ~100 GB of [L, L] probabilities)
        return {'skipped': f'seq {cfg["L"]}: the dense CPU oracle does not fit a bounded sample'}
    import oracle
    from oracle.params import portable_ids
    threads = host_cores()
    torch.set_num_threads(threads)
    hp = oracle.HParams(d_model=cfg['d'], num_heads=cfg['heads'], num_layers=cfg['layers'])
    params = {k: v.requires_grad_(True) for k, v in oracle.init_params(hp, 0, test_init=False).items()}
    L = cfg['L']

    def run(B):
        ids = torch.from_numpy(portable_ids((B, L), 11))
        ntok = torch.full((B,), L, dtype=torch.int64)
        eps = torch.randn(B, 1, 64)
        t0 = time.time()
        out = oracle.training_step(params, hp, ids, ntok, eps)
        out['loss'].backward()
        for p in params.values():
            p.grad = None
        return time.time() - t0

    run(2)
    # the config's own batch at seq 512 (C2: 64 x 512); longer sequences (C4/C5, ~10x the CPU work per sequence)
    # a batch of B/8 sequences, so the sample stays at 10-30 s of CPU time
    B = cfg['B'] if cfg['L'] <= 512 else max(1, cfg['B'] // 8)
    dt = run(B)
    return {'value': round(B * L / dt, 1), 'unit': 'tokens/s', 'cores': threads, 'kind': 'port',
            'sample': f'oracle/ (torch fp32 CPU restatement, golden-pinned) fwd+bwd of the {cfg["layers"]}L '
                      f'd{cfg["d"]} model on one full batch {B} x {L} tokens ({dt:.2f} s) after a batch-2 warm-up, '
                      f'{threads} threads (affinity mask capped by the cgroup CPU quota)'}


PARITY_MAX_SEQ = 16384


def parity_check(cfg, device):
    """GPU engine vs CPU oracle on the bench config's own model (layers, d_model, heads, seq) at batch 2 (batch 1
    from seq 2048 on, to bound the CPU time), same portable weights and injected noise, dropout off; plus the
    fp32-kernel-mode argmax reconstructions at z = mu against the oracle's. The sequence is capped at PARITY_MAX_SEQ:
    the oracle's attention is dense ([heads, L, L] f32 scores: 335 GB at the c2s100k length, over a box's host-memory
    cap), so the longest configurations check parity on the same model at PARITY_MAX_SEQ tokens."""
    import oracle
    from oracle.params import portable_ids, portable_normal
    from sparse_vae.engine import FlatParams, VAEEngine
    d, L = cfg['d'], min(cfg['L'], PARITY_MAX_SEQ)
    hp = oracle.HParams(d_model=d, num_heads=cfg['heads'], num_layers=cfg['layers'], kl_weight=0.7,
                        attn_window=cfg.get('window', 0))
    params = oracle.init_params(hp, 3)
    B = 2 if L < 2048 else 1
    ids = torch.from_numpy(portable_ids((B, L), 5))
    ntok = torch.full((B,), L, dtype=torch.int64)
    eps = torch.from_numpy(portable_normal(B * 64, 'eps', 3).reshape(B, 1, 64).astype('float32'))
    with torch.no_grad():
        ref = oracle.training_step(params, hp, ids, ntok, eps)
    flat = FlatParams(hp, device)
    for n in flat.offsets:
        flat.view(n).copy_(params[n])
    eng = VAEEngine(hp, flat)
    out = eng.forward(ids.to(device), ntok.to(device), eps=eps.to(device), dropout=0.0, kl_weight=0.7)
    loss, nll, kl = out['loss'].item(), out['nll'].item(), out['kl'].item()
    elbo, elbo_ref = -(nll + kl), -(ref['nll'].item() + ref['kl'].item())
    # argmax reconstructions at z = mu: fp32 kernel mode vs the CPU fp32 path
    from sparse_vae import kernels as K
    x = torch.empty(B * L, d, device=device)
    K.embedding_fwd(ids.to(torch.int32).to(device), flat.f('input_layer.0.weight'), x, B * L, d)
    mu = out['mu'].clone()
    am_gpu = eng.reconstruct_f32(x.view(B, L, d), mu)[:, :-1].argmax(-1).cpu()
    with torch.no_grad():
        xr = torch.nn.functional.embedding(ids, params['input_layer.0.weight'])
        am_ref = oracle.reconstruct(params, xr, mu.cpu().view(B, 1, 64), ids.eq(0), hp)[:, :-1].argmax(-1)
    seq = f'seq {L}' + (f' (the config\'s {cfg["L"]} capped for the dense CPU oracle)' if L < cfg['L'] else '')
    return {'config': f'{cfg["layers"]}L d{d} heads {cfg["heads"]} {seq} at batch {B}, dropout off, injected eps',
            'loss_gpu': loss, 'loss_cpu_ref': ref['loss'].item(),
            'loss_rel_err': abs(loss - ref['loss'].item()) / abs(ref['loss'].item()),
            'elbo_rel_err': abs(elbo - elbo_ref) / abs(elbo_ref), 'tolerance': 1e-3,
            'argmax_fp32_mode_agreement': (am_gpu == am_ref).float().mean().item()}


def _free_port():
    import socket
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def device_count_in_child(python=sys.executable):
    """GPUs visible to a fresh process. Queried in a child so the launcher itself never initialises HIP (a
    process that has must not fork ranks off)."""
    r = subprocess.run([python, '-c', 'import torch; print(torch.cuda.device_count())'],
                       capture_output=True, text=True, timeout=600)
    try:
        return int(r.stdout.strip().splitlines()[-1])
    except (ValueError, IndexError):
        return 0


def rank_env(rank, world, port, base=None):
    """The environment torch.distributed.run gives rank `rank` of a one-node job."""
    env = dict(os.environ if base is None else base)
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
               GROUP_RANK='0', MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')          # dmabuf IPC for RCCL (see the image notes)
    return env


def launch_ranks(world, child_argv, poll_s=0.2):
    """`python bench.py --gpus N` (N > 1) with no WORLD_SIZE in the environment: the reference's route to N GPUs is
    Lightning's `Trainer(gpus=N)` (train.py:63-64, 94), which spawns one DDP process per GPU. Do the same: start N
    child processes of `child_argv` with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set (one
    per GPU, RCCL over xGMI), wait for all of them, and return the first non-zero exit code (0 when all
    succeed). Rank 0 prints the JSON line on the inherited stdout; no other rank prints to stdout. If one rank
    fails, the others are terminated (they would wait forever in a collective)."""
    port = _free_port()
    procs = [subprocess.Popen(child_argv, env=rank_env(r, world, port)) for r in range(world)]
    rc = 0
    try:
        live = list(procs)
        while live:
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0 and rc == 0:
                    rc = code
                    print(f'bench.py: rank {procs.index(p)} exited with {code}; stopping the other ranks',
                          file=sys.stderr, flush=True)
                    for q in live:
                        q.terminate()
            time.sleep(poll_s)
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
                try:
                    p.wait(timeout=20)
                except subprocess.TimeoutExpired:
                    p.kill()
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=5)
    ap.add_argument('--config', default=None)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-parity', action='store_true')
    args = ap.parse_args()

    if args.gpus > 1 and 'WORLD_SIZE' not in os.environ:
        # launcher: this process never touches the GPU; it checks the device count in a child and starts one
        # rank per GPU
        n = device_count_in_child()
        # SVAE_BENCH_SHARE_GPUS=1 (rehearsal only, never a bench number): ranks share the visible GPUs round-robin,
        # so the N-rank launch path runs end to end on a 1-GPU box (with SVAE_DIST_BACKEND=gloo)
        share = os.environ.get('SVAE_BENCH_SHARE_GPUS') == '1'
        if n < args.gpus and not (share and n >= 1):
            print(f'bench.py: --gpus {args.gpus} needs {args.gpus} visible GPUs, this node has {n}',
                  file=sys.stderr, flush=True)
            sys.exit(3)
        sys.exit(launch_ranks(args.gpus, [sys.executable, '-u', os.path.abspath(__file__)] + sys.argv[1:]))

    world = int(os.environ.get('WORLD_SIZE', '1'))
    if world != args.gpus:
        print(f'bench.py: WORLD_SIZE={world} overrides --gpus {args.gpus}', file=sys.stderr, flush=True)
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if os.environ.get('SVAE_BENCH_SHARE_GPUS') == '1':
        local %= torch.cuda.device_count()
    torch.cuda.set_device(local)
    device = torch.device('cuda', local)
    if world > 1:
        # 'nccl' is RCCL on ROCm (the product path); SVAE_DIST_BACKEND=gloo only for the shared-GPU rehearsal
        backend = os.environ.get('SVAE_DIST_BACKEND', 'nccl')
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=device)
        else:
            dist.init_process_group(backend)
    cfg_name = args.config or 'c2'
    cfg = CONFIGS[cfg_name]

    model, opt, sched, batch = build(cfg, device)
    if world > 1:
        model.enable_data_parallel()
    eng = model._engine

    for _ in range(args.warmup):
        step(model, opt, sched, batch)

    # dominant-kernel timing: HIP events around every vocab-head GEMM launch of the timed steps
    probes = []
    eng.probe = probes
    comm = [] if world > 1 else None
    model.comm_probe = comm
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(model, opt, sched, batch)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    eng.probe = None
    model.comm_probe = None
    exposed = None
    if world > 1:
        t = torch.tensor([dt], device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = t.item()
        # exposed communication per step: the compute stream's wait for the gradient all-reduce past the end of the
        # backward (the buckets launched during the backward overlap it; what remains is this tail), max over ranks
        ex = sum(a.elapsed_time(b) for a, b in comm) / max(1, len(comm))
        te = torch.tensor([ex], device=device)
        dist.all_reduce(te, op=dist.ReduceOp.MAX)
        exposed = te.item()
    ms = dt / args.steps * 1e3
    tokens = cfg['B'] * cfg['L'] * world * args.steps
    value = tokens / dt
    fpt = flops_per_token(cfg['layers'], cfg['d'], cfg['L'], window=cfg.get('window', 0))
    fpt_causal = flops_per_token_causal(cfg['layers'], cfg['d'], cfg['L'], window=cfg.get('window', 0))
    loss = model.logged.get('train_nll')

    scaling = None
    if world > 1:
        # same-run N = 1 figure: every rank re-runs the K steps with the data-parallel gradient all-reduce off
        # (model._dp = None is exactly the single-GPU step); after the timed region, so it never enters `value`
        dp, model._dp = model._dp, None
        dist.barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            step(model, opt, sched, batch)
        torch.cuda.synchronize()
        d1 = torch.tensor([time.perf_counter() - t1], device=device)
        dist.all_reduce(d1, op=dist.ReduceOp.MAX)
        model._dp = dp
        single = cfg['B'] * cfg['L'] * args.steps / d1.item()
        scaling = {'value': round(value / (world * single), 4), 'single_gpu_tokens_per_s': round(single, 1),
                   'basis': f'same run: the {args.steps} steps re-timed on every rank with the gradient all-reduce '
                            f'off (the N=1 step, max over ranks); efficiency = value / (N x that rate)'}

    if rank == 0:
        T = cfg['B'] * cfg['L']
        head_ms = sum(a.elapsed_time(b) for a, b in probes) / max(1, len(probes))
        head_flops = 2.0 * T * cfg['d'] * V
        achieved = head_flops / (head_ms * 1e-3) / 1e12 if head_ms > 0 else None
        traffic = None
        pmc = os.path.join(ROOT, 'profiles', f'pmc_head_gemm_{cfg_name}.json')
        if os.path.exists(pmc):
            with open(pmc) as f:
                traffic = json.load(f).get('hbm_bytes_per_launch')
        res = {
            'metric': METRIC, 'value': round(value, 1), 'unit': 'tokens/s', 'n_gpus': world, 'steps': args.steps,
            'warmup': args.warmup, 'ms_per_step': round(ms, 3), 'higher_is_better': True, 'scaling': 'weak',
            'vs_baseline': None, 'dtype': 'bf16', 'data': 'synthetic (uniform ids in [3, 32768), [CLS] first, no padding; random-init weights)',
            'config': {'workload': f'{cfg_name}: TransformerVAE {cfg["layers"]}L d{cfg["d"]} heads {cfg["heads"]} seq {cfg["L"]}, '
                                   f'batch {cfg["B"]}/GPU, '
                                   + (f'sliding-window decoder attention (window {cfg["window"]} x 32)' if cfg.get('window')
                                      else 'dense attention')
                                   + ', dropout 0.1, fwd+bwd+allreduce+clip+RAdam',
                       'model': f'TransformerVAE-{cfg["layers"]}L-d{cfg["d"]}', 'global_batch': cfg['B'] * world,
                       'seq_len': cfg['L'], 'parallelism': f'dp{world}'},
            'model_tflops_per_gpu': round(value / world * fpt / 1e12, 1),
            'step_mfu': round(value / world * fpt / (PEAK_BF16_TFLOPS * 1e12), 4),
            'step_mfu_causal': round(value / world * fpt_causal / (PEAK_BF16_TFLOPS * 1e12), 4),
            'roofline': {'kernel': ('gemm256_kernel<false,false,SVAE_EPI_CE_PROB> (vocab head, stores P = exp(logit - '
                                    'label logit) + per-tile sums)' if eng.head_mode == 'prob' else
                                    'gemm256_kernel<false,false,SVAE_EPI_CE_STATS> (vocab head + CE stats)'),
                         'bound': 'mfma', 'achieved': round(achieved, 1) if achieved else None,
                         'peak': PEAK_BF16_TFLOPS, 'unit': 'TFLOP/s',
                         'frac': round(achieved / PEAK_BF16_TFLOPS, 4) if achieved else None,
                         'traffic': traffic, 'launch_ms': round(head_ms, 4), 'flops_per_launch': head_flops},
            'final_train_nll': round(loss.item(), 5) if torch.is_tensor(loss) else None,
        }
        if scaling is not None:
            res['scaling_efficiency'] = scaling
        if exposed is not None:
            res['exposed_comm_ms'] = {'value': round(exposed, 4), 'fraction_of_step': round(exposed / ms, 4),
                                      'basis': 'HIP events on the compute stream from the end of the backward to the '
                                               'last bucket all-reduce wait, mean over the timed steps, max over ranks'}
        if os.environ.get('SVAE_BENCH_SHARE_GPUS') == '1':
            res['rehearsal'] = (f'NOT a measurement: {world} ranks share {torch.cuda.device_count()} GPU(s), backend '
                                f'{os.environ.get("SVAE_DIST_BACKEND", "nccl")}')
        if world == 1 and not args.no_parity:
            try:
                res['parity'] = parity_check(cfg, device)
            except Exception as e:  # parity is reported, never allowed to kill the throughput line
                res['parity'] = {'error': repr(e)}
        if world == 1 and not args.no_cpu_baseline:
            res['cpu_baseline'] = cpu_baseline(cfg)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
