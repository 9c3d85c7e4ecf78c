"""Two-rank (gloo, one GPU) run of the train_twotower entry on the entry test's synthetic tables,
printing each rank's per-epoch metrics (diagnostic for tests/test_gpu_entry.py).
    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 tools/entry_dp_probe.py DIR [lazy]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'tests')]
os.environ.setdefault('RSYS_DIST_BACKEND', 'gloo')
os.environ['LOCAL_RANK'] = '0'
if len(sys.argv) > 2 and sys.argv[2] == 'lazy':
    os.environ['RSYS_LAZY_ROWS'] = '1'

import pathlib  # noqa: E402

import torch  # noqa: E402

import test_gpu_entry as te  # noqa: E402
from recommendsystemproject_amd.project.utils import training_utils as tu  # noqa: E402
from recommendsystemproject_amd.train_twotower import main  # noqa: E402

tmp = pathlib.Path(sys.argv[1])
tmp.mkdir(parents=True, exist_ok=True)
if int(os.environ.get('RANK', '0')) == 0:
    te._write_inputs(tmp, epochs=2, n_train=750)
import torch.distributed as dist  # noqa: E402
orig = tu.validate


def validate(*a, **k):
    loss, m = orig(*a, **k)
    print(f"rank {os.environ.get('RANK')} val_loss {loss:.5f} metrics {m}", flush=True)
    return loss, m


import recommendsystemproject_amd.train_twotower as tt  # noqa: E402
tt.validate = validate
if int(os.environ.get('WORLD_SIZE', '1')) > 1:
    import time
    while not (tmp / 'items.pkl').exists():
        time.sleep(0.2)
    time.sleep(1.0)
p = {k: str(tmp / v) for k, v in (('config', 'config.yaml'), ('meta', 'meta.yaml'), ('train', 'train.pkl'),
                                  ('val', 'val.pkl'), ('items', 'items.pkl'))}
model, best = main(p['config'], p['train'], p['val'], p['items'], p['meta'], checkpoint_dir=str(tmp / 'ckpt'),
                   device=torch.device('cuda:0'))
print('best', best, flush=True)
if dist.is_initialized():
    dist.destroy_process_group()
