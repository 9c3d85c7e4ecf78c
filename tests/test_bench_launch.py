"""bench.py --gpus N without torchrun (the driver's scaling command): the process becomes a
launcher of N rank processes (bench.launch_ranks) and itself never touches the GPU. CPU tests
with stub rank commands; the real two-rank run is tests/test_dist.py::test_bench_two_ranks_gloo_one_gpu
(-m gpu)."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_PARENT = r'''
import json, os, sys
sys.path.insert(0, {root!r})
sys.argv = ['bench.py', '--gpus', '{n}', '--steps', '1', '--warmup', '0']
import torch
import bench
stub = [sys.executable, '-c', {stub!r}]
orig = bench.launch_ranks
bench.launch_ranks = lambda n, argv: orig(n, argv, cmd=stub, poll_s=0.05)
code = 0
try:
    bench.main()
except SystemExit as e:
    code = e.code
# the launcher made no HIP call: no device context, the HIP library never loaded
print(json.dumps({{'parent_rc': code, 'cuda_initialized': torch.cuda.is_initialized(),
                  'hip_lib_loaded': bench._hip._LIB is not None}}))
'''

_RANK_OK = ("import os, json; print(json.dumps({k: os.environ[k] for k in "
            "('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'MASTER_ADDR', 'MASTER_PORT')}), flush=True)")
_RANK_FAILS = ("import os, sys, time\n"
               "if os.environ['RANK'] == '1': sys.exit(3)\n"
               "time.sleep(120)")


def _run_parent(n, stub, timeout=60):
    env = {k: v for k, v in os.environ.items() if k not in ('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'MASTER_PORT')}
    env['HIP_VISIBLE_DEVICES'] = ''
    src = _PARENT.format(root=ROOT, n=n, stub=stub)
    return subprocess.run([sys.executable, '-c', src], cwd=ROOT, env=env, capture_output=True, text=True,
                          timeout=timeout)


def test_launcher_starts_n_ranks_and_forwards_rank0():
    r = _run_parent(3, _RANK_OK)
    assert r.returncode == 0, r.stderr[-2000:]
    out = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith('{')]
    # stdout: rank 0's line (forwarded) then the parent's report; ranks 1, 2 went to stderr
    assert len(out) == 2, r.stdout
    rank0, parent = out
    assert rank0['RANK'] == '0' and rank0['LOCAL_RANK'] == '0' and rank0['WORLD_SIZE'] == '3'
    assert rank0['MASTER_ADDR'] == '127.0.0.1' and int(rank0['MASTER_PORT']) > 0
    others = [json.loads(ln) for ln in r.stderr.splitlines() if ln.startswith('{"RANK"')]
    assert sorted(o['RANK'] for o in others) == ['1', '2']
    assert all(o['MASTER_PORT'] == rank0['MASTER_PORT'] and o['WORLD_SIZE'] == '3' for o in others)
    assert parent == {'parent_rc': 0, 'cuda_initialized': False, 'hip_lib_loaded': False}


def test_launcher_fails_fast_when_a_rank_fails():
    t0 = time.time()
    r = _run_parent(2, _RANK_FAILS)
    assert time.time() - t0 < 40  # rank 0 (sleeping 120 s) was stopped, not waited for
    parent = json.loads(r.stdout.strip().splitlines()[-1])
    assert parent['parent_rc'] == 3 and not parent['cuda_initialized']
    assert 'rank 1 exited with 3' in r.stderr


def test_bench_gpus_must_match_world(monkeypatch):
    """Under torchrun, --gpus must equal WORLD_SIZE (the line's n_gpus is the process group's)."""
    src = ("import sys; sys.path.insert(0, %r); sys.argv = ['bench.py', '--gpus', '2']\n"
           "import bench\n"
           "bench.rdist.init_from_env = lambda: None\n"
           "bench.main()\n") % ROOT
    env = dict(os.environ, WORLD_SIZE='1', HIP_VISIBLE_DEVICES='')
    r = subprocess.run([sys.executable, '-c', src], cwd=ROOT, env=env, capture_output=True, text=True, timeout=60)
    assert r.returncode != 0 and '--gpus 2 but the process group has 1 ranks' in r.stderr
