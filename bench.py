"""Benchmark: two-tower DSSM training samples/sec on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2] [--batch 4096]
    torchrun --nproc-per-node N bench.py --gpus N ...       (one process per GPU, RCCL)

`python bench.py --gpus N` (N > 1, no torchrun) launches the N rank processes itself
(launch_ranks) and forwards rank 0's line.

Workload (BASELINE.json configs[1]): MovieLens-1M-schema DSSM + Transformer sequence encoder,
seq_len 50, d_model 64, per-GPU batch 4096, dropout as configured, temperature from the config,
Adam + clip_grad_norm_(1.0). Synthetic MovieLens-shaped batches (synth.py), resident in HBM
before timing. A "step" = zero_grad + forward + in-batch loss + backward + [RCCL all-reduce]
+ clip + Adam, captured as two hipGraphs (fwd/bwd, optimizer) and replayed.
Prints ONE JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import faulthandler
import json
import os
import sys
import time

# Hardware queues per process (GPU_MAX_HW_QUEUES) are left at the box's setting, HIP's default 4,
# which is also what the training entry runs with; the effective value is recorded in the line.
# Measured (tools/gpu_hwq_ab.sh, round 4): 8 queues made the C2 step 1.42 -> 3.0-3.2 ms (C3 equal).

import torch  # noqa: E402
import torch.distributed as dist
import yaml

ROOT = os.path.dirname(os.path.abspath(__file__))
T_START = time.time()
sys.path.insert(0, ROOT)

from recommendsystemproject_amd import dist as rdist  # noqa: E402
from recommendsystemproject_amd import _hip  # noqa: E402
from recommendsystemproject_amd import synth  # noqa: E402
from recommendsystemproject_amd import precision  # noqa: E402
from recommendsystemproject_amd.flat import ensure_flat  # noqa: E402
from recommendsystemproject_amd.optim import Adam  # noqa: E402
from recommendsystemproject_amd.profiling import KernelTimer, PmcBracket  # noqa: E402
from recommendsystemproject_amd.project.models.TwoTower.GenericTower import GenericTower  # noqa: E402
from recommendsystemproject_amd.project.models.TwoTower.TwoTowerModel import TwoTowerModel  # noqa: E402
from recommendsystemproject_amd.project.utils.training_utils import backward_seed, extract_item_id  # noqa: E402

PEAK_F32_TFLOPS = 157.3   # MI355X f32 (vector = f32-input MFMA) peak, MI355X_MICROARCH.md
PEAK_BF16_TFLOPS = 2500.0  # MI355X dense bf16 MFMA peak (no sparsity), MI355X_MICROARCH.md
PEAK_HBM_GBS = 8000.0     # HBM3E spec
HBM_MEASURED_GBS = 6290.0  # MI355X_MICROARCH.md: measured float4 copy (79 % of spec); replaced by
                           # this run's own copy measurement (measure_peaks)
# v_exp_f32 issues in 8 cycles per wave on one SIMD (MI355X_MICROARCH.md cycle constants):
# 64 lanes / 8 cycles x 4 SIMDs x 256 CUs x 2.4 GHz
PEAK_EXP_PER_S = 64 / 8 * 4 * 256 * 2.4e9
CE_ENTRIES = ('rs_inbatch_ce_fused_fwd', 'rs_inbatch_ce_fused_bwd', 'rs_inbatch_ce_fused_fwd_uib',
              'rs_inbatch_ce_fused_bwd_uib', 'rs_inbatch_ce_fused_f32_fwd', 'rs_inbatch_ce_fused_f32_bwd')
SOFTMAX_ENTRIES = ('rs_attn_fwd', 'rs_attn_bwd') + CE_ENTRIES


WORKLOADS = {
    'c3': 'synthetic 10M-item vocab DSSM (emb 128, pooled 50-long history, lazy-exact Adam tables)',
    'c5': 'synthetic 100M-item vocab DSSM (emb 64, lazy-exact Adam tables)',
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=None,
                    help='ranks (one process per GPU). Without torchrun\'s WORLD_SIZE, N > 1 makes this '
                         'process a launcher of N rank processes (launch_ranks); under torchrun it must '
                         'equal WORLD_SIZE')
    ap.add_argument('--steps', type=int, default=100)  # 100 x 1.24 ms at C2: averages out the box's step-to-step noise
    ap.add_argument('--warmup', type=int, default=5)
    ap.add_argument('--config', default='c2')
    ap.add_argument('--batch', type=int, default=None, help='per-GPU batch (default: config)')
    ap.add_argument('--dropout', default='config', choices=['config', '0'])
    ap.add_argument('--no-graph', action='store_true')
    ap.add_argument('--dtype', default='config', choices=['config', 'fp32', 'bf16'],
                    help='compute dtype of the GEMMs (bf16: bf16 MFMA, fp32 accumulate / master weights); '
                         'config: bf16 for c2 (BASELINE configs[1] is quoted in bf16), c3 (the fused bf16 '
                         'in-batch CE) and c5 (its L = 200 encoder runs on the bf16 MFMA attention), fp32 '
                         'otherwise; --dtype fp32 is the parity precision')
    ap.add_argument('--hard-negatives', type=int, default=0,
                    help='N sampled hard negatives per row, materialised from a device item catalog '
                         'each step (one grouped item-tower pass)')
    ap.add_argument('--zipf', type=float, default=None, help='Zipf(alpha) ids instead of uniform (C3 variant)')
    ap.add_argument('--batches', type=int, default=8,
                    help='distinct resident batches cycled through by the timed steps')
    ap.add_argument('--extra', default=None,
                    help='comma-separated further workloads reported in the same JSON line under '
                         '"extra", each NAME or NAME:DTYPE (default when --config is c2: c3 at fp32, the '
                         "reference's precision and the credited C3 number, and c3:bf16 beside it)")
    ap.add_argument('--prof-markers', action='store_true',
                    help='profiling runs: an rs_prof_marker dispatch right before and after every timed '
                         'loop, so tools/prof_summary.py can bracket a rocprofv3 kernel trace to the '
                         'timed steps')
    ap.add_argument('--cpu-baseline-seconds', type=float, default=15.0)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--pmc-bracket', default=None, metavar='ENTRY|auto',
                    help='profiling pass only: one eager step with every call of ENTRY (auto: the '
                         'dominant entry point) between rs_prof_marker dispatches, for '
                         'rocprofv3 --pmc (tools/pmc_traffic.py); prints a JSON line and exits')
    ap.add_argument('--traffic', default='auto',
                    help='PMC traffic summary (tools/pmc_traffic.py output) for roofline.traffic; '
                         'auto: profiles/traffic_<config>_<dtype>.json when it matches this run')
    ap.add_argument('--cpu-worker', nargs=2, default=None, metavar=('SPEC', 'OUT'), help=argparse.SUPPRESS)
    a = ap.parse_args()
    if a.extra is None:
        if a.config == 'c2' and a.batch is None and not a.zipf:
            # N = 1 (the driver's BENCH line): every BASELINE workload that fits one GPU -- C3 at fp32
            # (credited) and bf16, C3 with Zipf(1.05) ids, C5 with 10 hard negatives; N > 1 (the
            # scaling runs): C3 data-parallel = configs[3] (C4), both precisions
            one = int(os.environ.get('WORLD_SIZE', '1')) == 1
            a.extra = 'c3:fp32,c3:bf16' + (',c3_zipf:fp32,c5:fp32,c5:bf16' if one else '')
        else:
            a.extra = ''
    return a


def run_key(args, B, name=None, dtype=None, zipf=None, hard_negatives=None):
    """What a PMC traffic summary must match to be reported on this run's roofline."""
    return {'config': name or args.config, 'dtype': dtype or args.dtype, 'batch': B,
            'dropout': args.dropout, 'hard_negatives': args.hard_negatives if hard_negatives is None else hard_negatives,
            'zipf': zipf}


def load_traffic(args, B, entry, name, dtype, zipf, hard_negatives, suffix=''):
    """roofline.traffic: HBM bytes per launch of `entry` from a committed rocprofv3 --pmc summary
    (FETCH_SIZE and WRITE_SIZE in separate passes, gfx950 read correction; tools/pmc_traffic.py),
    used only when it was collected on this same workload and entry point."""
    path = args.traffic
    if path == 'none':
        return None
    if path == 'auto':  # Zipf-id runs of a config have their own files (traffic_c3_zipf_fp32_gather.json)
        path = os.path.join(ROOT, 'profiles', f'traffic_{name}{"_zipf" if zipf else ""}_{dtype}{suffix}.json')
    if not os.path.exists(path):
        return None
    tr = json.load(open(path))
    if tr.get('entry') != entry or tr.get('run') != run_key(args, B, name, dtype, zipf, hard_negatives):
        return None
    out = {k: tr[k] for k in ('hbm_bytes_per_launch', 'hbm_read_bytes_per_launch',
                              'write_bytes_per_launch', 'alg_bytes_per_launch', 'launches') if k in tr}
    out['traffic_over_alg'] = round(tr['hbm_bytes_per_launch'] / max(tr['alg_bytes_per_launch'], 1), 3)
    out['source'] = os.path.relpath(path, ROOT)
    return out


CPU_VOCAB_CAP = 10_000_000  # host-memory bound of the CPU baseline's tables (C5: 100M rows)


def _cap_vocab(cfg, cap):
    """cfg with every table capped at `cap` rows (ids are drawn within the vocab, so the sample
    stays well-formed); returns (cfg, capped?)."""
    import copy
    cfg = copy.deepcopy(cfg)
    capped = False

    def walk(o):
        nonlocal capped
        if isinstance(o, dict):
            if isinstance(o.get('vocab_size'), int) and o['vocab_size'] > cap:
                o['vocab_size'] = cap
                capped = True
            for v in o.values():
                walk(v)
        elif isinstance(o, list):
            for v in o:
                walk(v)
    walk(cfg)
    return cfg, capped


def _oracle_rate(cfg, seconds, B, dropout, min_steps=1):
    """Samples/s of the oracle's training step on the bench's own first batches (seed 1000 + i,
    the GPU rank 0's), timed after one warm-up step, for about `seconds` and at least `min_steps`
    steps."""
    from oracle.twotower_oracle import OracleTrainer, model_state_shapes
    import copy
    cfg = copy.deepcopy(cfg)
    if dropout == '0':
        for t in cfg['two_tower'].values():
            t['dropout'] = 0.0
            t.get('transformer_parameters', {})['dropout'] = 0.0
    maps = {'user': synth.tower_layout(cfg['two_tower']['user_tower']),
            'item': synth.tower_layout(cfg['two_tower']['item_tower'])}
    shapes = {k: s for k, s, _ in model_state_shapes(cfg)}
    tr = OracleTrainer(cfg, synth.make_state(shapes, seed=1), lr=cfg['train']['learning_rate'], dropout=None)
    batches = [synth.batch_to_torch(synth.make_batch(cfg, B, seed=1000 + i)) for i in range(2)]
    T = cfg['train']['temperature']
    tr.step(batches[0], maps, temperature=T)  # warm-up
    n, t0 = 0, time.perf_counter()
    while True:
        tr.step(batches[n % 2], maps, temperature=T)
        n += 1
        el = time.perf_counter() - t0
        if (el >= seconds and n >= min_steps) or n >= 200:
            break
    return n * B / el, n, el


def cpu_baseline(cfg, seconds, B, min_steps=10, legs=('config', '0')):
    """The oracle (CPU restatement of the reference step, fp32) on a bounded sample of the same
    workload: the configured batch B and the GPU's own batches, dropout as configured and p = 0
    (half the time each), on the torch threads of the box's CPU share. Tables above CPU_VOCAB_CAP
    rows are capped (the oracle's dense Adam over a 100M x 64 table and its state exceed the
    box's host-memory limit); the sample says so."""
    cfg, capped = _cap_vocab(cfg, CPU_VOCAB_CAP)
    rate, n, el = _oracle_rate(cfg, seconds / len(legs), B, 'config', min_steps)
    rate0 = n0 = el0 = None
    if '0' in legs:  # the p = 0 leg: half the steps
        rate0, n0, el0 = _oracle_rate(cfg, seconds / len(legs), B, '0', max(3, min_steps // 2))
    model = None
    try:
        for line in open('/proc/cpuinfo'):
            if line.startswith('model name'):
                model = line.split(':', 1)[1].strip()
                break
    except OSError:
        pass
    return {'value': round(rate, 1), 'unit': 'samples/s', 'cores': torch.get_num_threads(),
            'kind': 'port', 'value_p0': None if rate0 is None else round(rate0, 1),
            'sample': f'{n} steps x batch {B} (the GPU run\'s first batches; oracle, fp32, dropout as '
                      f'configured), {el:.1f} s' + ('' if rate0 is None else f'; p = 0 leg: {n0} steps, {el0:.1f} s') +
                      (f'; tables capped at {CPU_VOCAB_CAP:,} rows (host memory)' if capped else '') +
                      f'; {torch.get_num_threads()} torch threads of {os.cpu_count()} host cores (the '
                      f'GPU box\'s CPU share is 16 threads)',
            'threads': torch.get_num_threads(), 'nproc': os.cpu_count(), 'cpu_model': model, 'steps': n,
            'seconds': round(el, 1), 'batch': B}


def cpu_worker(spec_path, out_path):
    """The CPU baselines of one bench run, in a child process started before the GPU is touched
    (a plain CPU python: it never initialises HIP). It waits for the parent's 'go' on stdin,
    sent once every GPU workload has been timed, so the two legs never share the host cores.
    Writes {key: cpu_baseline} as each finishes."""
    spec = json.load(open(spec_path))
    if not sys.stdin.readline():  # EOF: the parent is gone (or failed) before its go -- no orphan run
        return
    res = {}
    for job in spec['jobs']:
        cfg = yaml.safe_load(open(os.path.join(ROOT, 'configs', f"{job['config']}.yaml")))
        if job.get('zipf'):
            cfg.setdefault('synthetic', {})['zipf'] = job['zipf']
        try:
            res[job['key']] = cpu_baseline(cfg, job['seconds'], job['batch'], job['min_steps'], tuple(job['legs']))
        except Exception as e:  # a baseline must not cost the line
            res[job['key']] = {'error': repr(e)[:300]}
        json.dump(res, open(out_path + '.tmp', 'w'))
        os.replace(out_path + '.tmp', out_path)


def start_cpu_worker(jobs):
    """-> (process, result path). Started before any HIP call of this process: the child is a
    plain CPU python (it never touches the GPU)."""
    import subprocess
    import tempfile
    d = tempfile.mkdtemp(prefix='rsys_cpu_')
    spec, out = os.path.join(d, 'spec.json'), os.path.join(d, 'out.json')
    json.dump({'jobs': jobs}, open(spec, 'w'))
    env = dict(os.environ, HIP_VISIBLE_DEVICES='', CUDA_VISIBLE_DEVICES='', ROCR_VISIBLE_DEVICES='')
    proc = subprocess.Popen([sys.executable, os.path.abspath(__file__), '--cpu-worker', spec, out], env=env,
                            stdin=subprocess.PIPE, stdout=subprocess.DEVNULL,
                            stderr=open(os.path.join(d, 'err.log'), 'w'))
    return proc, out


def release_cpu_worker(proc):
    """The GPU timing is over: the CPU baselines may start."""
    try:
        proc.stdin.write(b'go\n')
        proc.stdin.close()
    except OSError:
        pass


def collect_cpu_worker(proc, out, timeout):
    """Wait for the CPU baselines (a progress line every 30 s: a silent run looks hung)."""
    t0 = time.time()
    while True:
        try:
            proc.wait(timeout=30)
            break
        except Exception:
            pass
        if time.time() - t0 > timeout:
            print('[bench] CPU baselines timed out', file=sys.stderr, flush=True)
            proc.kill()
            proc.wait()
            break
        try:
            done = sorted(json.load(open(out)))
        except Exception:
            done = []
        print(f'[bench] waiting for the CPU baselines ({time.time() - t0:.0f} s; done: {done})', file=sys.stderr,
              flush=True)
    try:
        return json.load(open(out))
    except Exception:
        return {}


def measure_peaks(dev, copy_bytes=1 << 31, reps=5):
    """This box's own peaks, measured in the same run (report against the datasheet
    AND the measured figures): a float4 streaming copy of 2 GiB (HBM read + write bytes over the
    event time, best of `reps`) and back-to-back v_mfma_f32_32x32x16_bf16 on every SIMD
    (csrc/peaks.hip)."""
    from recommendsystemproject_amd import _hip
    st = torch.cuda.current_stream()
    src = torch.empty(copy_bytes // 4, dtype=torch.float32, device=dev).fill_(1.0)
    dst = torch.empty_like(src)
    best_copy = 0.0
    for _ in range(reps + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        _hip.call('rs_peak_copy', src.data_ptr(), dst.data_ptr(), copy_bytes, st.cuda_stream)
        e1.record(st)
        e1.synchronize()
        best_copy = max(best_copy, 2.0 * copy_bytes / (e0.elapsed_time(e1) * 1e-3) / 1e9)
    del src, dst
    blocks, iters = 2048, 2048  # 8 waves per SIMD on 256 CUs
    out = torch.empty(blocks * 4, dtype=torch.float32, device=dev)
    flops = int(_hip.lib().rs_peak_mfma_flops(blocks, iters))
    best_mfma = 0.0
    for _ in range(reps + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        _hip.call('rs_peak_mfma', out.data_ptr(), blocks, iters, st.cuda_stream)
        e1.record(st)
        e1.synchronize()
        best_mfma = max(best_mfma, flops / (e0.elapsed_time(e1) * 1e-3) / 1e12)
    torch.cuda.empty_cache()
    return {'hbm_copy_GBs': round(best_copy, 1), 'bf16_mfma_TFLOPs': round(best_mfma, 1),
            'how': 'float4 copy of 2 GiB (read + write bytes), best of 5; back-to-back '
                   'v_mfma_f32_32x32x16_bf16, 2048 x 256-thread workgroups, best of 5 (csrc/peaks.hip)'}


def _copy_pairs(dst, src, out):
    if isinstance(src, torch.Tensor):
        out.append((dst, src))
    elif isinstance(src, dict):
        for k, v in src.items():
            _copy_pairs(dst[k], v, out)
    elif isinstance(src, list):
        for d, v in zip(dst, src):
            _copy_pairs(d, v, out)


_COPY_PLANS = {}


def _copy_into(dst, src):
    """Next resident batch -> the static input slot the captured graphs read (device copies, as
    a loader writing the next batch would), all in one rs_copy_many launch. The pointer arrays of
    a (slot, batch) pair are built once: the per-step host work is one ctypes call, so the host
    stays ahead of the replayed graphs."""
    import ctypes as C
    key = (id(dst), id(src))
    plan = _COPY_PLANS.get(key)
    if plan is None:
        pairs = []
        _copy_pairs(dst, src, pairs)
        plan = []
        for k in range(0, len(pairs), 32):
            part = pairs[k:k + 32]
            for d, s in part:
                assert d.is_contiguous() and s.is_contiguous() and d.nbytes == s.nbytes and d.dtype == s.dtype
            n = len(part)
            srcs = (C.c_void_p * n)(*[s.data_ptr() for _, s in part])
            dsts = (C.c_void_p * n)(*[d.data_ptr() for d, _ in part])
            nb = (C.c_int64 * n)(*[s.nbytes for _, s in part])
            plan.append((n, srcs, dsts, nb, C.addressof(srcs), C.addressof(dsts), C.addressof(nb), pairs))
        _COPY_PLANS[key] = plan
    st = torch.cuda.current_stream().cuda_stream
    for n, _s, _d, _n, ps, pd, pn, _keep in plan:
        _hip.call('rs_copy_many', n, ps, pd, pn, st)


def _clone(b):
    if isinstance(b, torch.Tensor):
        return b.clone()
    if isinstance(b, dict):
        return {k: _clone(v) for k, v in b.items()}
    if isinstance(b, list):
        return [_clone(v) for v in b]
    return b


def load_cfg(name, args):
    cfg = yaml.safe_load(open(os.path.join(ROOT, 'configs', f'{name}.yaml')))
    if args.dropout == '0':
        for t in cfg['two_tower'].values():
            t['dropout'] = 0.0
            t.get('transformer_parameters', {})['dropout'] = 0.0
    return cfg


# Lazy-exact Adam's per-row work (csrc/lookup.hip, sparse.hip; adam.h), priced per distinct row
# of a sorted call (flat.profile_call_rows: [(D, lookups, distinct rows)] of the priced steps):
#   catch-up: p, m, v read, p written (weight decay 0: the moments are replayed in registers),
#             `last` read + written;
#   Adam    : p, g, m, v read, p, m, v written, g re-zeroed, `last` read + written;
#   sqnorm  : g read.
LAZY_ROW_BYTES = {
    'rs_sorted_catchup': lambda rows: sum(r * (16.0 * D + 16.0) for D, _, r in rows),
    'rs_sorted_adam_batch': lambda rows: sum(r * (32.0 * D + 16.0) for D, _, r in rows),
    'rs_sorted_sqnorm_batch': lambda rows: sum(r * 4.0 * D for D, _, r in rows),
}
# round 5: the dense region rides in the first sorted batch's launch (+ 28 B / 4 B per dense param)
LAZY_ROW_BYTES['rs_sorted_adam_batch_dense'] = LAZY_ROW_BYTES['rs_sorted_adam_batch']
LAZY_ROW_BYTES['rs_sorted_sqnorm_batch_dense'] = LAZY_ROW_BYTES['rs_sorted_sqnorm_batch']
DENSE_BYTES_PER_PARAM = {'rs_adam_step': 28.0, 'rs_sorted_adam_batch_dense': 28.0, 'rs_sorted_sqnorm_batch_dense': 4.0}
LAZY_ROW_BYTES['rs_sorted_catchup_batch'] = LAZY_ROW_BYTES['rs_sorted_catchup']  # round 6: one launch per gather
LAZY_ENTRIES = ('rs_lookup_sort', 'rs_sorted_catchup', 'rs_sorted_catchup_batch', 'rs_segsum',
                'rs_segsum_batch', 'rs_sorted_sqnorm_batch', 'rs_sorted_adam_batch', 'rs_sorted_sqnorm_batch_dense',
                'rs_sorted_adam_batch_dense')


def optimizer_roofline(summ, rows, flat_numel, dense_numel, ms_step, args, B, name, dtype, zipf, hard_negatives):
    """the reference's optimizer sweeps every parameter, 28 B/param/step ('dense
    equivalent': C3 2.69B params -> 75 GB); lazy-exact Adam moves the touched rows only. Reports
    both, and the lazy chain (sort, catch-up, segment sum, clip partials, sorted Adam) and the
    dense Adam over the non-table parameters as bytes / event time against 8 TB/s, with the
    PMC traffic of the catch-up and the Adam step where collected on this workload. None
    without large tables."""
    if not rows:
        return None
    steps = 3.0  # the instrumented pass
    ent = {}
    tot_ms = tot_by = 0.0
    for k in LAZY_ENTRIES + ('rs_adam_step',):
        if k not in summ:
            continue
        ms = summ[k]['ms'] / steps
        by = (LAZY_ROW_BYTES[k](rows) if k in LAZY_ROW_BYTES else summ[k]['bytes']) / steps
        if k == 'rs_adam_step':
            by = 0.0
        by += DENSE_BYTES_PER_PARAM.get(k, 0.0) * dense_numel  # the dense region [0, dense_numel)
        ent[k] = {'ms_per_step': round(ms, 4), 'bytes_per_step': round(by),
                  'GBs': round(by / (ms * 1e-3) / 1e9, 1) if ms > 0 else None,
                  'frac': round(by / (ms * 1e-3) / (PEAK_HBM_GBS * 1e9), 4) if ms > 0 else None}
        tr = load_traffic(args, B, k, name, dtype, zipf, hard_negatives, suffix='_' + k.replace('rs_', ''))
        if tr:
            ent[k]['traffic'] = tr['hbm_bytes_per_launch']
            ent[k]['traffic_detail'] = tr
        tot_ms += ms
        tot_by += by
    dense_eq = 28.0 * flat_numel
    distinct = sum(r for _, _, r in rows) / steps
    lookups = sum(n for _, n, _ in rows) / steps
    return {'dense_equivalent_bytes_per_step': round(dense_eq),
            'dense_equivalent_ms_at_8TBs': round(dense_eq / (PEAK_HBM_GBS * 1e9) * 1e3, 3),
            'params': flat_numel,
            'lazy_bytes_per_step': round(tot_by), 'lazy_ms_per_step': round(tot_ms, 4),
            'lazy_GBs': round(tot_by / (tot_ms * 1e-3) / 1e9, 1) if tot_ms > 0 else None,
            'frac': round(tot_by / (tot_ms * 1e-3) / (PEAK_HBM_GBS * 1e9), 4) if tot_ms > 0 else None,
            'lazy_share_of_step': round(tot_ms / ms_step, 3),
            'bytes_ratio_dense_over_lazy': round(dense_eq / max(tot_by, 1.0), 1),
            'table_rows_stepped_per_step': round(distinct), 'table_lookups_per_step': round(lookups),
            'entries': ent,
            'model': '28 B/param dense (SURVEY 8d); per distinct row: catch-up 16D+16 B, Adam 32D+16 B, '
                     'clip partials 4D B; sort and segment sum as profiling.WORK; event time with the '
                     'towers serial (instrumented pass)'}


def run_workload(args, name, dtype, zipf, hard_negatives, rank, world, dev, cpu_seconds, peaks=None):
    """Build the model of workload `name`, time args.steps steps (after args.warmup) cycling through
    args.batches distinct resident batches, profile one instrumented pass. Returns the result dict
    on rank 0 (None elsewhere); with args.pmc_bracket, prints the bracket line and returns None."""
    cfg = load_cfg(name, args)
    if rank == 0:
        print(f'[bench] {name} {dtype}: setting up', file=sys.stderr, flush=True)
    if zipf:
        cfg.setdefault('synthetic', {})['zipf'] = zipf
    precision.set_compute_dtype(dtype)
    B = args.batch or int(cfg['train']['batch_size'])
    T = float(cfg['train']['temperature'])
    maps = {'user': synth.tower_layout(cfg['two_tower']['user_tower']),
            'item': synth.tower_layout(cfg['two_tower']['item_tower'])}

    torch.manual_seed(0)
    big = max(int(f.get('vocab_size', 0)) for t in cfg['two_tower'].values()
              for f in (t.get('sparse_features') or []) + (t.get('sequence_features') or [])) >= 10 ** 7
    if big:  # 10M-100M-row tables: initialise on the device (CPU init of 25 GB tables takes minutes)
        with torch.device(dev):
            model = TwoTowerModel(GenericTower(cfg, 'user_tower'), GenericTower(cfg, 'item_tower'),
                                  maps['user'], maps['item'])
    else:
        model = TwoTowerModel(GenericTower(cfg, 'user_tower'), GenericTower(cfg, 'item_tower'),
                              maps['user'], maps['item']).to(dev)
    model.train()
    n_sharded = sum(t.shard is not None for t in ensure_flat(model).lazy)  # W >= 4: row-sharded tables
    rdist.broadcast_model(model)
    opt = Adam(model.parameters(), lr=float(cfg['train']['learning_rate']))
    opt.grad_scale = 1.0 / world
    # K distinct batches resident in HBM (per rank), cycled through by every step: the lazy-Adam
    # catch-up replays real skipped steps and the gathered rows are not one cache-resident set
    K = max(1, args.batches)
    batches = [synth.batch_to_torch(synth.make_batch(cfg, B, seed=1000 + 97 * rank + i), dev)
               for i in range(K)]
    batch = _clone(batches[0])  # the static slot the graphs read
    ids = extract_item_id(batch['item_tower'])
    catalog = None
    neg_sets = neg_ids = None
    if hard_negatives:
        # synthetic item catalog (id column = row, other features random) and uniformly sampled
        # negative ids (one set per resident batch); the N item-tower dicts are materialised
        # inside every step
        from recommendsystemproject_amd.project.utils.hard_negatives import ItemCatalog
        item_cfg = cfg['two_tower']['item_tower']
        V = int(item_cfg['sparse_features'][0]['vocab_size'])
        g = torch.Generator(device=dev).manual_seed(7 + rank)
        cols = [f for f in item_cfg['sparse_features'] if 'pooling' not in f]
        sparse = torch.stack([torch.arange(V, device=dev, dtype=torch.int32) if i == 0 else
                              torch.randint(1, int(f['vocab_size']), (V,), device=dev, generator=g, dtype=torch.int32)
                              for i, f in enumerate(cols)], 1)
        seqc = {f['name']: torch.randint(0, int(f['vocab_size']), (V, 3), device=dev, generator=g, dtype=torch.int32)
                for f in item_cfg['sparse_features'] if 'pooling' in f}
        catalog = ItemCatalog(sparse=sparse, sequence=seqc, device=dev)
        neg_sets = [torch.randint(1, V, (B, hard_negatives), device=dev, generator=g) for _ in range(K)]
        neg_ids = neg_sets[0].clone()

    def fwd_bwd():
        opt.zero_grad()
        if catalog is not None:
            batch['hard_negatives'] = catalog.materialize(neg_ids)
        U, I, H = model(batch)
        loss = model.compute_loss(U, I, item_ids=ids, hard_neg_emb=H, temperature=T)
        with rdist.overlap(model):  # N > 1: each tower's all-reduce starts inside the backward
            loss.backward(backward_seed(loss))
        return loss

    def opt_step():
        opt.step(clip_max_norm=1.0)

    def allreduce():
        if world > 1:
            rdist.allreduce_gradients(model, opt)

    counter = [0]

    def next_batch():
        i = counter[0] % K
        counter[0] += 1
        _copy_into(batch, batches[i])
        if neg_sets is not None:
            neg_ids.copy_(neg_sets[i], non_blocking=True)

    # eager warm-up (also allocates Adam state), then capture
    # eager warm-up; a PMC bracket step comes after every resident batch has been stepped once, so
    # its large-table rows are (batches - 1) steps stale like the timed steps' (the catch-up's
    # replay, its reads of the moments, are then those of the timed run)
    n_warm = max(2, min(args.warmup, 3))
    if args.pmc_bracket:
        n_warm = max(n_warm, args.batches)
    for _ in range(n_warm):
        next_batch()
        fwd_bwd()
        allreduce()
        opt_step()
    torch.cuda.synchronize()
    if rank == 0:
        print(f'[bench] {name} {dtype}: {n_warm} eager warm-up steps done ({time.time() - T_START:.0f} s)',
              file=sys.stderr, flush=True)
    if args.pmc_bracket:
        target = args.pmc_bracket
        if target == 'auto':
            with KernelTimer() as kt:
                next_batch()
                fwd_bwd()
                allreduce()
                opt_step()
            target = max(kt.summary().items(), key=lambda kv: kv[1]['ms'])[0]
        torch.cuda.synchronize()
        next_batch()
        from recommendsystemproject_amd import flat as _flat
        _flat.PROFILE_CALLS = []
        with PmcBracket(target) as pb:
            fwd_bwd()
            allreduce()
            opt_step()
        torch.cuda.synchronize()
        rows = _flat.profile_call_rows(_flat.PROFILE_CALLS)
        _flat.PROFILE_CALLS = None
        if target in LAZY_ROW_BYTES:  # per-row work: priced from this step's distinct-row counts
            pb.bytes = (LAZY_ROW_BYTES[target](rows) +
                        DENSE_BYTES_PER_PARAM.get(target, 0.0) * ensure_flat(model).dense_numel)
        if rank == 0:
            print(json.dumps({'pmc_bracket': target, 'launches': pb.launches,
                              'alg_bytes_per_launch': pb.bytes / max(pb.launches, 1),
                              'alg_flops_per_launch': pb.flops / max(pb.launches, 1),
                              'run': run_key(args, B, name, dtype, zipf, hard_negatives)}))
        return None
    graphs = None
    # N > 1 (RCCL): the gradient all-reduce and the large tables' exchange are captured with the
    # backward -- their host-side bookkeeping (this step's lookup calls, the buckets started in
    # the backward) runs once, at capture, and every replay re-runs all of their collectives.
    # Host-staged gloo collectives (ranks sharing one GPU) cannot be captured: eager steps.
    if world > 1 and dist.get_backend() != 'nccl':
        args.no_graph = True
    if not args.no_graph:
        try:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                fwd_bwd()
                allreduce()
                opt_step()
            torch.cuda.current_stream().wait_stream(s)
            # thread_local: the RCCL process group's watchdog thread polls its work events while
            # this thread captures; a global-mode capture would be invalidated by those queries.
            # One graph for the whole step (RSYS_BENCH_GRAPHS=2: forward+backward and the optimizer
            # as two, round 3's split, which left ~10 us between them)
            if os.environ.get('RSYS_BENCH_GRAPHS', '1') == '2':
                g1, g2 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
                with torch.cuda.graph(g1, capture_error_mode='thread_local'):
                    loss_static = fwd_bwd()
                    allreduce()
                with torch.cuda.graph(g2, capture_error_mode='thread_local'):
                    opt_step()
            else:
                g1, g2 = torch.cuda.CUDAGraph(), None
                with torch.cuda.graph(g1, capture_error_mode='thread_local'):
                    loss_static = fwd_bwd()
                    allreduce()
                    opt_step()
            graphs = (g1, g2, loss_static)
            if rank == 0:
                print(f'[bench] {name} {dtype}: step captured', file=sys.stderr, flush=True)
        except Exception as e:  # eager fallback keeps the same kernels
            print(f'[bench] graph capture failed ({e!r}); running eagerly', file=sys.stderr)
            graphs = None

    def step():
        next_batch()
        if graphs is not None:
            graphs[0].replay()
            if graphs[1] is not None:
                graphs[1].replay()
            return graphs[2]
        loss = fwd_bwd()
        allreduce()
        opt_step()
        return loss

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    if args.prof_markers:
        from recommendsystemproject_amd import _hip as _h
        _h.call('rs_prof_marker', 7, torch.cuda.current_stream().cuda_stream)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    t_issue = time.perf_counter() - t0  # host time to enqueue the steps (the GPU waits if it is ~el)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if args.prof_markers:
        _h.call('rs_prof_marker', 8, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
    el_t = torch.tensor([el], device=dev)
    if world > 1:
        dist.all_reduce(el_t, op=dist.ReduceOp.MAX)
    el = float(el_t.item())
    final_loss = float(loss.item())
    if rank == 0:
        print(f'[bench] {name} {dtype}: {1e3 * el / args.steps:.3f} ms/step; instrumented passes next',
              file=sys.stderr, flush=True)
    model.check_errors()  # device error flags (bad ids, NaN embeddings) of the timed steps

    # roofline of the dominant kernel: HIP events on the launch stream, eager instrumented steps.
    # A spin kernel first gives the host a head start: the launches (Python + ctypes, slower than
    # the small tower kernels themselves) then queue up behind it and the GPU runs them back to
    # back, so an event pair times its kernel and not the host's launch latency.
    # The towers run serially here (RSYS_TOWER_STREAMS=0): each event pair then times its kernel
    # alone, not its kernel sharing the GPU with the other tower's.
    torch.cuda.synchronize()
    tower_streams = os.environ.get('RSYS_TOWER_STREAMS')
    os.environ['RSYS_TOWER_STREAMS'] = '0'
    torch.cuda._sleep(int(2.4e9 * 0.03))  # ~30 ms at the 2.4 GHz shader clock
    from recommendsystemproject_amd import flat as _flat
    _flat.PROFILE_CALLS = []  # the large tables' sorted calls of these steps (distinct-row counts)
    with KernelTimer() as kt:
        for _ in range(3):
            next_batch()
            fwd_bwd()
            allreduce()
            opt_step()
    lazy_rows = _flat.profile_call_rows(_flat.PROFILE_CALLS)
    _flat.PROFILE_CALLS = None
    fl_ = ensure_flat(model)
    flat_numel = sum(int(p.numel()) for p in fl_.params)  # every parameter (full tables)
    dense_numel = fl_.dense_numel
    if tower_streams is None:
        del os.environ['RSYS_TOWER_STREAMS']
    else:
        os.environ['RSYS_TOWER_STREAMS'] = tower_streams
    summ = kt.summary()
    dom_name, dom = max(summ.items(), key=lambda kv: kv[1]['ms'])
    # the dominant entry point's MFMA peak: bf16 MFMA in the bf16 compute mode (its products,
    # attention's included: they run on v_mfma_*_bf16), f32 else
    peak_mfma = PEAK_BF16_TFLOPS if dtype == 'bf16' else PEAK_F32_TFLOPS
    flop_bound = dom['flops'] / max(dom['bytes'], 1.0) > peak_mfma * 1e12 / (PEAK_HBM_GBS * 1e9)
    avg_ms = dom['ms'] / dom['launches']
    if flop_bound:
        achieved = dom['flops'] / dom['launches'] / (avg_ms * 1e-3) / 1e12
        roof = {'bound': 'mfma', 'achieved': round(achieved, 3), 'peak': peak_mfma, 'unit': 'TFLOP/s'}
    else:
        achieved = dom['bytes'] / dom['launches'] / (avg_ms * 1e-3) / 1e9
        roof = {'bound': 'hbm', 'achieved': round(achieved, 1), 'peak': PEAK_HBM_GBS, 'unit': 'GB/s'}
    roof['frac'] = round(roof['achieved'] / roof['peak'], 4)
    if peaks:  # against this box's own measured peak too
        pm = peaks['hbm_copy_GBs'] if roof['unit'] == 'GB/s' else \
            (peaks['bf16_mfma_TFLOPs'] if peak_mfma == PEAK_BF16_TFLOPS else None)
        if pm:
            roof['peak_measured'] = pm
            roof['frac_of_measured'] = round(roof['achieved'] / pm, 4)
    if dom.get('exps'):  # softmax kernels: their exponentials against the v_exp issue rate
        roof['valu_exp'] = {'exps_per_launch': dom['exps'] / dom['launches'],
                            'achieved_per_s': dom['exps'] / (dom['ms'] * 1e-3),
                            'peak_per_s': PEAK_EXP_PER_S,
                            'frac': round(dom['exps'] / (dom['ms'] * 1e-3) / PEAK_EXP_PER_S, 4)}
    roof['traffic'] = None
    tr = load_traffic(args, B, dom_name, name, dtype, zipf, hard_negatives)
    if tr is not None:
        roof['traffic'] = tr['hbm_bytes_per_launch']
        roof['traffic_detail'] = tr
    roof['kernel'] = dom_name
    roof['avg_launch_ms'] = round(avg_ms, 4)
    roof['share_of_step'] = round(dom['ms'] / sum(v['ms'] for v in summ.values()), 3)
    # whole-step roofline: max(sum bytes / HBM peak, sum flops / f32 MFMA peak) of the
    # instrumented entry points' algorithmic work, over the measured step time
    step_flops = sum(v['flops'] for v in summ.values()) / 3
    step_bytes = sum(v['bytes'] for v in summ.values()) / 3
    bound_ms = max(step_bytes / (PEAK_HBM_GBS * 1e9),
                   step_flops / ((PEAK_BF16_TFLOPS if dtype == 'bf16' else PEAK_F32_TFLOPS) * 1e12)) * 1e3
    step_roof = {'flops_per_step': round(step_flops), 'bytes_per_step': round(step_bytes),
                 'bound_ms': round(bound_ms, 4), 'frac': round(bound_ms / (el / args.steps * 1e3), 4)}
    # the embedding gather against the HBM roofline (north_star: >= 70 % on the gather), against the
    # 8 TB/s spec and against the measured float4-copy bandwidth (report both)
    gather_roof = {}
    # the table gradient = the scatter of ordinary tables (rs_gather_bwd) + the sorted segment
    # sum of the large ones (rs_segsum); the sort itself runs in the forward (rs_lookup_sort)
    # catchup_gather: the lazy tables' forward unit -- the catch-up that brings a call's distinct rows
    # current, then the gather that reads them (priced by their own algorithmic bytes, both kernels'
    # event time)
    groups = {'rs_gather_fwd': ('rs_gather_fwd', 'rs_gather_fwd_lazy'),
              'table_grad': ('rs_gather_bwd', 'rs_segsum', 'rs_segsum_batch'),
              'catchup_gather': ('catchup', 'rs_gather_fwd', 'rs_gather_fwd_lazy')}
    gs = dict(summ)  # the groups' entries, with the forward catch-up merged
    cu = [gs[k] for k in ('rs_sorted_catchup', 'rs_sorted_catchup_batch') if k in gs]
    if cu and lazy_rows:  # the forward catch-up (one launch per gather since round 6), priced per
        # distinct row (LAZY_ROW_BYTES), as optimizer_roofline
        gs['catchup'] = {'ms': sum(x['ms'] for x in cu), 'bytes': LAZY_ROW_BYTES['rs_sorted_catchup'](lazy_rows)}
    for k, members in groups.items():
        if k == 'catchup_gather' and 'catchup' not in gs:
            continue
        ms = [gs[m] for m in members if m in gs]
        g = {'ms': sum(x['ms'] for x in ms), 'bytes': sum(x['bytes'] for x in ms)}
        if g['ms'] > 0:
            gbs = g['bytes'] / (g['ms'] * 1e-3) / 1e9
            gather_roof[k] = {'achieved': round(gbs, 1), 'peak': PEAK_HBM_GBS, 'unit': 'GB/s',
                              'frac': round(gbs / PEAK_HBM_GBS, 4),
                              'frac_of_measured_copy': round(gbs / (peaks or {}).get('hbm_copy_GBs', HBM_MEASURED_GBS), 4),
                              'bytes_per_step': round(g['bytes'] / 3),
                              'ms_per_step': round(g['ms'] / 3, 4), 'entries': list(members)}
            if k == 'catchup_gather' and lazy_rows:
                # the catch-up's other bound: its replay of the skipped zero-gradient Adam steps is VALU
                # work (adam.h adam_replay_zero: per element pair and step 9 packed fp32 operations at 4
                # cycles and 4 transcendentals at 8 -- MI355X_MICROARCH.md issue costs -- on 64 lanes),
                # modelled with every distinct row (batches - 1) steps stale, the bench's cycle
                el_steps = sum(D * r for D, _, r in lazy_rows) / 3 * max(args.batches - 1, 0)
                valu_ms = el_steps * 34.0 / 64 / (1024 * 2.4e9) * 1e3
                ms_c = gs['catchup']['ms'] / 3
                gather_roof[k]['catchup_valu_model'] = {
                    'element_steps_per_step': round(el_steps), 'valu_bound_ms': round(valu_ms, 4),
                    'catchup_ms_per_step': round(ms_c, 4), 'frac': round(valu_ms / ms_c, 4) if ms_c > 0 else None,
                    'model': '34 SIMD cycles per element and replayed step, 1024 SIMDs x 2.4 GHz, '
                             'rows (batches - 1) steps stale'}
            if k == 'rs_gather_fwd':  # PMC traffic of the gather (profiles/traffic_<cfg>_<dt>_gather.json)
                tr = load_traffic(args, B, 'rs_gather_fwd', name, dtype, zipf, hard_negatives, suffix='_gather')
                gather_roof[k]['traffic'] = tr['hbm_bytes_per_launch'] if tr else None
                if tr:
                    gather_roof[k]['traffic_detail'] = tr

    # the batch similarity (U I^T inside the fused in-batch CE) against the MFMA peak of its
    # operands (bf16, or f32 in fp32 mode) (north_star: MFMA utilisation on the batch-dot)
    batch_dot = {}
    for k in CE_ENTRIES:
        if k in summ and summ[k]['ms'] > 0:
            g = summ[k]
            tf = g['flops'] / (g['ms'] * 1e-3) / 1e12
            pk = PEAK_F32_TFLOPS if '_f32_' in k else PEAK_BF16_TFLOPS
            batch_dot[k] = {'achieved': round(tf, 1), 'peak': pk, 'unit': 'TFLOP/s',
                            'frac': round(tf / pk, 4),
                            'exp_frac': round(g['exps'] / (g['ms'] * 1e-3) / PEAK_EXP_PER_S, 4),
                            'flops_per_launch': round(g['flops'] / g['launches']),
                            'avg_launch_ms': round(g['ms'] / g['launches'], 4)}

    # the softmax kernels against both their bounds: the bf16 MFMA (their products) and the
    # v_exp issue rate (one exponential per (query, key) / logit per direction)
    softmax = {}
    for k in SOFTMAX_ENTRIES:
        if k in summ and summ[k]['ms'] > 0 and summ[k]['exps'] > 0:
            g = summ[k]
            sec = g['ms'] * 1e-3
            softmax[k] = {'ms_per_step': round(g['ms'] / 3, 4),
                          'mfma_frac': round(g['flops'] / sec / 1e12 / (PEAK_BF16_TFLOPS if dtype == 'bf16' else PEAK_F32_TFLOPS), 4),
                          'exp_frac': round(g['exps'] / sec / PEAK_EXP_PER_S, 4)}

    opt_roof = optimizer_roofline(summ, lazy_rows, flat_numel, dense_numel, ms_step=el / args.steps * 1e3,
                                  args=args, B=B, name=name, dtype=dtype, zipf=zipf, hard_negatives=hard_negatives)
    used_graph = graphs is not None
    _COPY_PLANS.clear()  # the plans hold this workload's batch tensors (and key on their ids)
    if graphs is not None:  # the graphs (and the RCCL kernels they hold at N > 1) go first
        torch.cuda.synchronize()
        for g in graphs[:2]:
            if g is not None:
                g.reset()
    del model, opt, batches, batch, graphs, catalog
    torch.cuda.empty_cache()
    cpu = None

    if rank != 0:
        return None
    samples = world * B * args.steps
    tp = cfg['two_tower']['user_tower'].get('transformer_parameters', {})
    has_seq = bool(cfg['two_tower']['user_tower'].get('sequence_features'))
    return {
        'metric': 'training samples/sec (user-item pairs) at batch 4096; 1/2/4/8 MI355X',
        'value': round(samples / el, 1), 'unit': 'samples/s', 'n_gpus': world, 'steps': args.steps,
        'warmup': args.warmup, 'ms_per_step': round(el / args.steps * 1e3, 3),
        'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None, 'dtype': dtype,
        'data': f'synthetic (MovieLens-1M-shaped ids, seeded numpy PCG64, {K} distinct batches '
                f'resident in HBM, cycled)',
        'config': {'workload': f'{name}: ' + WORKLOADS.get(name, 'MovieLens-1M DSSM') +
                   (f' + Transformer seq encoder (seq_len {tp.get("max_seq_len")}, d={cfg["two_tower"]["user_tower"]["embedding_dim"]})' if has_seq else ''),
                   'global_batch': world * B, 'per_gpu_batch': B,
                   'seq_len': tp.get('max_seq_len') if has_seq else None,
                   'dropout': args.dropout, 'parallelism': f'dp{world}',
                   'hip_graph': used_graph, 'final_loss': round(final_loss, 5),
                   'host_issue_ms_per_step': round(t_issue / args.steps * 1e3, 3),
                   'ids': f'zipf({zipf})' if zipf else 'uniform',
                   'hard_negatives': hard_negatives, 'resident_batches': K,
                   'gpu_max_hw_queues': os.environ.get('GPU_MAX_HW_QUEUES', 'unset (HIP default 4)'),
                   'row_sharded_tables': n_sharded},
        'roofline': roof,
        'gather_roofline': gather_roof,
        'batch_dot_roofline': batch_dot or None,
        'softmax_roofline': softmax or None,
        'step_roofline': step_roof,
        'optimizer_roofline': opt_roof,
        'cpu_baseline': cpu,
        'kernel_ms_per_step': {k: round(v['ms'] / 3, 4) for k, v in sorted(summ.items(), key=lambda kv: -kv[1]['ms'])},
        '_gemm_shapes': kt.gemm_shapes() if os.environ.get('RSYS_BENCH_DETAIL') else None,
    }


def _cpu_jobs(args):
    """The CPU baselines of this run (rank 0, N = 1): the primary workload (dropout as configured
    and a p = 0 leg), each extra workload's config once (one leg), and C1 (BASELINE configs[0]).
    >= 10 steps per leg (the p = 0 leg 5; C5 5 -- its oracle step at L = 200 with 10M-row tables
    takes ~25 s on the host). C3-Zipf reuses C3's: the oracle's dense step costs the same for any
    ids. The legs run one after another in one child process, after the GPU timing (~4 min)."""
    jobs, seen = [], set()

    def add(key, config, primary=False):
        if config in seen:
            return
        seen.add(config)
        c = yaml.safe_load(open(os.path.join(ROOT, 'configs', f'{config}.yaml')))
        B = args.batch or int(c['train']['batch_size'])
        big = config == 'c5'
        jobs.append({'key': key, 'config': config, 'zipf': args.zipf if primary else None, 'batch': B,
                     'seconds': 5.0 if big else args.cpu_baseline_seconds,
                     'min_steps': 5 if big else 10, 'legs': ['config', '0'] if primary and not big else ['config']})
    add(args.config, args.config, primary=True)
    for ex in [e for e in (args.extra or '').split(',') if e]:
        nm = ex.partition(':')[0]
        add('c3' if nm == 'c3_zipf' else nm, 'c3' if nm == 'c3_zipf' else nm)
    add('c1', 'c1')
    return jobs


def _frac(d, *path):
    for k in path:
        if not isinstance(d, dict) or d.get(k) is None:
            return None
        d = d[k]
    return d


def _cpu_short(c):
    if not c or 'error' in c:
        return c
    return {k: c.get(k) for k in ('value', 'unit', 'cores', 'kind', 'threads', 'nproc', 'steps', 'seconds',
                                  'batch', 'value_p0', 'sample')}


def _extra_short(r):
    if 'error' in r:
        return {'error': r['error'][:200]}
    g = r.get('gather_roofline') or {}
    return {'value': r['value'], 'ms_per_step': r['ms_per_step'], 'dtype': r['dtype'],
            'workload': r['config']['workload'].split(':')[0],
            'roofline_frac': _frac(r, 'roofline', 'frac'), 'roofline_kernel': _frac(r, 'roofline', 'kernel'),
            'gather_frac': _frac(g, 'rs_gather_fwd', 'frac'),
            'catchup_gather_frac': _frac(g, 'catchup_gather', 'frac'),
            'catchup_valu_frac': _frac(g, 'catchup_gather', 'catchup_valu_model', 'frac'),
            'step_roofline_frac': _frac(r, 'step_roofline', 'frac'),
            'cpu_baseline_value': _frac(r, 'cpu_baseline', 'value'),
            'cpu_baseline_steps': _frac(r, 'cpu_baseline', 'steps'),
            'cpu_baseline_of': r.get('cpu_baseline_of', r['config']['workload'].split(':')[0])}


def compact_line(out):
    """The stdout line: the contract's fields, the dominant kernel's roofline without its PMC
    detail, the CPU baseline's numbers, and per extra workload its headline numbers only (the
    whole record is the stderr 'bench_detail' object). Kept well under 8 KB."""
    keys = ('metric', 'value', 'unit', 'n_gpus', 'steps', 'warmup', 'ms_per_step', 'higher_is_better', 'scaling',
            'vs_baseline', 'dtype', 'data')
    line = {k: out[k] for k in keys}
    cfg = out['config']
    line['config'] = {k: cfg.get(k) for k in ('workload', 'global_batch', 'per_gpu_batch', 'seq_len', 'dropout',
                                             'parallelism', 'hip_graph', 'ids', 'hard_negatives',
                                             'resident_batches', 'row_sharded_tables')}
    line['roofline'] = {k: v for k, v in out['roofline'].items() if k not in ('traffic_detail', 'valu_exp')}
    g = out.get('gather_roofline') or {}
    line['gather_roofline'] = {k: {'frac': v.get('frac'), 'achieved': v.get('achieved'), 'ms_per_step': v.get('ms_per_step'),
                                   'traffic': v.get('traffic')} for k, v in g.items()}
    for k, v in g.items():
        if v.get('catchup_valu_model'):
            line['gather_roofline'][k]['catchup_valu_frac'] = v['catchup_valu_model']['frac']
    line['step_roofline'] = out.get('step_roofline')
    line['cpu_baseline'] = _cpu_short(out.get('cpu_baseline'))
    c1 = out.get('c1_cpu_baseline')
    line['c1_cpu_baseline'] = {'value': c1.get('value'), 'steps': c1.get('steps'), 'batch': c1.get('batch')} \
        if c1 and 'error' not in c1 else c1
    pk = out.get('peaks_measured') or {}
    line['peaks_measured'] = {k: pk.get(k) for k in ('hbm_copy_GBs', 'bf16_mfma_TFLOPs')}
    if out.get('extra'):
        line['extra'] = {k: _extra_short(v) for k, v in out['extra'].items()}
    line['wall_s'] = out.get('wall_s')
    line['detail'] = 'stderr: {"bench_detail": ...}'
    return line


def _free_port():
    import socket
    with socket.socket() as sk:
        sk.bind(('127.0.0.1', 0))
        return sk.getsockname()[1]


def launch_ranks(n, argv, cmd=None, poll_s=0.5):
    """`bench.py --gpus N` without torchrun: this process starts N rank processes of itself (one
    per GPU, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set as torchrun sets them)
    and never touches the GPU itself -- it imports torch (no HIP call) and makes no torch.cuda
    call, so no rank is a fork or exec of a process that initialised HIP. Rank 0's stdout (the
    JSON line) is this process's stdout; the other ranks' stdout and every rank's stderr go to
    stderr. If a rank fails, the others are stopped (their process groups) and the exit code is
    the first failure's. `cmd`: the rank command (default: this script with `argv`)."""
    import signal
    import subprocess
    cmd = cmd or [sys.executable, '-u', os.path.abspath(__file__)] + list(argv)
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK='0', MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
        procs.append(subprocess.Popen(cmd, env=env, stdout=None if r == 0 else sys.stderr,
                                      start_new_session=True))
    rc = 0
    failed = None
    while True:
        alive = 0
        for r, p in enumerate(procs):
            code = p.poll()
            if code is None:
                alive += 1
            elif code != 0 and failed is None:
                failed, rc = r, code
        if failed is not None or alive == 0:
            break
        time.sleep(poll_s)
    if failed is not None:
        print(f'[bench] rank {failed} exited with {rc}; stopping the other ranks', file=sys.stderr, flush=True)
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGTERM)
                except OSError:
                    pass
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
                p.wait()
        rc = rc if rc > 0 else 1  # a signal death (negative) still fails the launcher
    return rc


def main():
    faulthandler.enable()  # a crash prints the Python stack of every thread
    args = parse()
    if args.cpu_worker:
        cpu_worker(*args.cpu_worker)
        return
    if (args.gpus or 1) > 1 and 'WORLD_SIZE' not in os.environ:
        # the driver's `python bench.py --gpus N`: be the launcher of N ranks (before any HIP call)
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    env_world = int(os.environ.get('WORLD_SIZE', '1'))
    if args.gpus is not None and args.gpus != env_world:  # before the CPU worker or any HIP call
        raise SystemExit(f'bench.py: --gpus {args.gpus} but the process group has {env_world} ranks')
    cpu_s = 0.0 if args.no_cpu_baseline else args.cpu_baseline_seconds
    worker = None
    if int(os.environ.get('WORLD_SIZE', '1')) == 1 and cpu_s > 0 and not args.pmc_bracket:
        # before any HIP call of this process: the CPU baselines run beside the GPU timing
        worker = start_cpu_worker(_cpu_jobs(args))
    rdist.init_from_env()
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    assert args.gpus is None or args.gpus == world
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if os.environ.get('RSYS_DIST_BACKEND') == 'gloo':  # rehearsal: ranks share the box's GPUs
        local %= max(torch.cuda.device_count(), 1)
    dev = torch.device(f'cuda:{local}')
    torch.cuda.set_device(dev)
    if args.dtype == 'config':
        args.dtype = 'bf16' if args.config in ('c2', 'c3', 'c5') else 'fp32'
    peaks = None if args.pmc_bracket else measure_peaks(dev)
    out = run_workload(args, args.config, args.dtype, args.zipf, args.hard_negatives, rank, world, dev,
                       cpu_s, peaks)
    if args.pmc_bracket:
        _teardown()
        return
    extras = {}
    order = [args.config]
    for ex in [e for e in (args.extra or '').split(',') if e]:
        # the other headline workloads in the same line (BASELINE configs[2] = C3; at N > 1 the
        # same run is configs[3] = C4, C3 data-parallel). NAME:DTYPE; the reference computes in
        # fp32, so an fp32 entry is reported under NAME and another precision under NAME_DTYPE
        name, _, ex_dtype = ex.partition(':')
        ex_dtype = ex_dtype or ('bf16' if name in ('c2', 'c3', 'c5') else 'fp32')
        key = name if ex_dtype == 'fp32' else f'{name}_{ex_dtype}'
        if (name, ex_dtype) == (args.config, args.dtype):
            continue
        zipf = 1.05 if name == 'c3_zipf' else None  # C3 with Zipf(1.05) ids
        cfg_name = 'c3' if name == 'c3_zipf' else name
        # the previous workload's model, optimizer state, batches and graph pools are released
        # before this one allocates (C5's 100M-row tables need ~200 GB of the 288)
        import gc
        gc.collect()
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        if rank == 0:
            print(f'[bench] {torch.cuda.memory_allocated(dev) / 2**30:.1f} GiB still allocated before {key}',
                  file=sys.stderr, flush=True)
        try:
            r = run_workload(args, cfg_name, ex_dtype, zipf, 10 if name == 'c5' else 0, rank, world, dev, 0.0,
                             peaks)
        except Exception as e:  # an extra workload must not cost the headline line
            import traceback
            traceback.print_exc(file=sys.stderr)
            extras[key] = {'error': repr(e)[:400]}
            r = None
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
        order.append(key)
        if r is not None:
            extras[key] = {k: r[k] for k in ('value', 'unit', 'ms_per_step', 'dtype', 'config', 'roofline',
                                             'gather_roofline', 'batch_dot_roofline', 'softmax_roofline',
                                             'step_roofline', 'optimizer_roofline', 'cpu_baseline',
                                             'kernel_ms_per_step')}
            if ex_dtype != 'fp32':
                extras[key]['note'] = (f'{ex_dtype} compute mode, beside the fp32 entry "{name}" (the '
                                       "reference's precision)")
    if worker is not None:
        # every GPU workload is timed: the CPU baselines run now, alone on the host cores; C1 =
        # BASELINE configs[0], the reference's CPU-runnable case (demo schema without the sequence
        # encoder, batch 256)
        print(f'[bench] GPU legs done ({time.time() - T_START:.0f} s); CPU baselines next', file=sys.stderr,
              flush=True)
        release_cpu_worker(worker[0])
        cpu = collect_cpu_worker(*worker, timeout=900)
        if rank == 0:
            out['cpu_baseline'] = cpu.get(args.config)
            for key in extras:
                nm = key.rsplit('_bf16', 1)[0] if key.endswith('_bf16') else key
                nm = 'c3' if nm == 'c3_zipf' else nm
                if 'error' not in extras[key]:
                    # one oracle run per config: the oracle computes in fp32 with a dense step whose
                    # cost does not depend on the ids, so the bf16 and Zipf entries share it
                    extras[key]['cpu_baseline'] = cpu.get(nm)
                    if nm != key:
                        extras[key]['cpu_baseline_of'] = nm
            out['c1_cpu_baseline'] = cpu.get('c1')
    if rank == 0:
        out['peaks_measured'] = peaks
        if args.prof_markers:
            out['prof_marker_order'] = order
        shapes = out.pop('_gemm_shapes', None)
        if shapes:
            shp = sorted(shapes.items(), key=lambda kv: -kv[1][0])
            print(json.dumps({'gemm_shapes_ms_per_step': [
                [list(k), round(v[0] / 3, 4), round(v[2] / (v[0] * 1e-3) / 1e12, 2) if v[0] else 0]
                for k, v in shp[:24]]}), file=sys.stderr)
        if extras:
            out['extra'] = extras
        out['wall_s'] = round(time.time() - T_START, 1)
        # the full record (per-kernel times, every roofline object, PMC traffic details) on stderr;
        # stdout carries ONE compact line the driver parses (round 4's 23 KB line was not parsed)
        print(json.dumps({'bench_detail': out}), file=sys.stderr, flush=True)
        print(json.dumps(compact_line(out)), flush=True)
    _teardown()


def _teardown():
    """Every captured graph (they hold RCCL kernels of the communicator at N > 1) is released and
    the device drained before the process group goes: ncclCommDestroy waits for the graphs that
    still use the communicator (round 5, gpurun_out/r5_b_rccl.log: a hang at exit otherwise)."""
    import gc
    gc.collect()
    if torch.cuda.is_initialized():
        torch.cuda.synchronize()
    if dist.is_initialized():
        if dist.get_world_size() > 1:
            dist.barrier()
        if torch.cuda.is_initialized():
            torch.cuda.synchronize()
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
