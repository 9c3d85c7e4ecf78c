"""train_twotower.py on the HIP path -- the reference's training entry (train_twotower.py:17-218)
with the same config.yaml / metadata_config.yaml schema, the same loop and the same checkpoint.

    python -m recommendsystemproject_amd.train_twotower [--config config.yaml] \
        [--train ./data/cleaned/train_set.pkl] [--val ./data/cleaned/val_set.pkl] \
        [--items ./data/cleaned/item_set.pkl] [--metadata-config metadata_config.yaml]
    torchrun --nproc-per-node N -m recommendsystemproject_amd.train_twotower ...   (data parallel)

What changes against the reference, and why:
* the loaders are the device loaders (DeviceLoader.py: the reference's collate on the GPU, same
  batch dicts, same DataLoader(shuffle=True) order), built from the same pickled DataFrames
  (or from a saved ColumnarDataset directory);
* the optimizer is optim.Adam (same arguments and state_dict layout as torch.optim.Adam; large
  tables stepped lazily and exactly, the clip fused);
* under torchrun each rank trains on its shard of every epoch's order (batch-parallel, SURVEY
  §8e), gradients are exchanged inside train_one_epoch, rank 0 writes the checkpoints.
The epoch loop, Recall@10 early stopping with `patience`, and the checkpoint dict (keys epoch,
model_state_dict, optimizer_state_dict, train_loss, val_loss, metrics, user_mapping,
item_mapping, config) are the reference's, so a checkpoint written here loads into the
reference's modules (state_dict keys are the reference's; lazy tables are flushed on save).
"""
from __future__ import annotations

import argparse
import os
from pathlib import Path

import torch
import torch.distributed as dist

from recommendsystemproject_amd import dist as rdist
from recommendsystemproject_amd.optim import Adam
from recommendsystemproject_amd.project.models.TwoTower.GenericTower import GenericTower
from recommendsystemproject_amd.project.models.TwoTower.TwoTowerModel import TwoTowerModel
from recommendsystemproject_amd.project.utils.config_utils import file_loader
from recommendsystemproject_amd.project.utils.DeviceLoader import (ColumnarDataset, DeviceCombinedLoader,
                                                                    DeviceTowerLoader)
from recommendsystemproject_amd.project.utils.training_utils import (build_user_history, train_one_epoch,
                                                                     validate)


def _read_table(path):
    """The reference reads pickled DataFrames (train_twotower.py:36, 61); a directory is a saved
    ColumnarDataset (the on-disk columnar format)."""
    if os.path.isdir(path):
        return ColumnarDataset.load(path)
    import pandas as pd
    return pd.read_pickle(path)  # the user's own data files, as the reference reads them


class _ShardedLoader:
    """Rank r of W takes every W-th batch of the epoch (the global batch is W x batch_size). The
    wrapped loader must draw the same order on every rank (dist.sync_seed) and drop its short last
    batch (drop_last): every rank's batch then has the same size, as the all-gathers of the
    lazy-table exchange require."""

    def __init__(self, loader, rank, world):
        self.loader, self.rank, self.world = loader, rank, world

    def __len__(self):
        return len(self.loader) // self.world  # equal on every rank (0 if fewer batches than ranks)

    def __iter__(self):
        n = len(self)
        for k, b in enumerate(self.loader):
            if k // self.world >= n:
                break
            if k % self.world == self.rank:
                yield b

    def get_feature_mappings(self):
        return self.loader.get_feature_mappings()


def main(config_path='config.yaml', train_data_path='./data/cleaned/train_set.pkl',
         val_data_path='./data/cleaned/val_set.pkl', item_data_path='./data/cleaned/item_set.pkl',
         metadata_config_path='metadata_config.yaml', checkpoint_dir='./checkpoints', epochs=None,
         device=None):
    """train_twotower.main (train_twotower.py:17-218). Returns (model, best_recall)."""
    rdist.init_from_env()
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    config = file_loader(config_path)
    if device is None:
        device = torch.device(f"cuda:{int(os.environ.get('LOCAL_RANK', '0'))}")
    torch.cuda.set_device(device)
    print(f'Using device: {device}')
    bs = config['train']['batch_size']

    if world > 1:
        rdist.sync_seed()  # one epoch order (and one model init) for every rank
    print('Setting up training dataloader...')
    train_df = _read_table(train_data_path)
    train_loader = DeviceCombinedLoader(config, train_df, batch_size=bs, shuffle=True, device=device,
                                        drop_last=world > 1)
    if world > 1:
        train_loader = _ShardedLoader(train_loader, rank, world)
    print('Setting up validation dataloader...')
    val_df = _read_table(val_data_path)
    val_loader = DeviceCombinedLoader(config, val_df, batch_size=bs, shuffle=False, device=device)
    print('Setting up item index dataloader...')
    item_loader = DeviceTowerLoader(config, _read_table(item_data_path), 'item_tower', batch_size=bs,
                                    shuffle=False, device=device)
    metadata = file_loader(metadata_config_path)
    val_metadata_loader = DeviceCombinedLoader(metadata, val_df, batch_size=bs, shuffle=False, device=device)
    meta_item = metadata.get('two_tower').get('item_tower').get('metadata_fields')
    meta_user = metadata.get('two_tower').get('user_tower').get('metadata_fields')
    user_history = build_user_history(train_df, user_col=meta_user, item_col=meta_item) \
        if not isinstance(train_df, ColumnarDataset) else None

    mappings = train_loader.get_feature_mappings()
    user_mapping, item_mapping = mappings['user'], mappings['item']
    print('\nFeature mappings:')
    print(f"  User sparse features: {list(user_mapping['sparse'].keys())}")
    print(f"  Item sparse features: {list(item_mapping['sparse'].keys())}")

    print('\nCreating model...')
    model = TwoTowerModel(GenericTower(config, 'user_tower'), GenericTower(config, 'item_tower'),
                          user_feature_mapping=user_mapping, item_feature_mapping=item_mapping).to(device)
    rdist.broadcast_model(model)
    print(f'Model created with {sum(p.numel() for p in model.parameters()):,} parameters')
    optimizer = Adam(model.parameters(), lr=config['train']['learning_rate'])

    num_epochs = int(epochs or config['train']['epochs'])
    temperature = config['train']['temperature']
    patience = config['train'].get('patience', 8)
    best_recall = 0.0
    patience_counter = 0
    print(f'\nStarting training for {num_epochs} epochs...')
    print(f'Temperature: {temperature}, Patience: {patience}')
    for epoch in range(1, num_epochs + 1):
        print(f"\n{'=' * 70}\nEpoch {epoch}/{num_epochs}\n{'=' * 70}")
        avg_train_loss = train_one_epoch(model=model, loader=train_loader, optimizer=optimizer, device=device,
                                         log_every_n_batches=100, epoch=epoch, temperature=temperature)
        # data parallel: rank 0's BatchNorm running statistics everywhere (DDP's broadcast_buffers),
        # so every rank validates the same model; the decisions below are rank 0's
        rdist.broadcast_buffers(model)
        movie_id_col_idx = item_mapping['sparse'].get('movie_id_enc', 0)
        avg_val_loss, metrics = validate(model=model, loader=val_loader, item_loader=item_loader,
                                         meta_data_loader=val_metadata_loader, device=device, epoch=epoch,
                                         k_list=[10, 20, 50], item_id_feature='movie_id_enc',
                                         item_id_type='sparse', item_id_col_idx=movie_id_col_idx,
                                         log_embeddings=True, user_history=user_history)
        current_recall = rdist.broadcast_scalar(metrics[10])
        if current_recall > best_recall:
            best_recall = current_recall
            patience_counter = 0
            save_path = Path(checkpoint_dir) / f'best_model_epoch_{epoch}.pt'
            # every rank: state_dict() gathers row-sharded tables (a collective)
            ckpt = {'epoch': epoch, 'model_state_dict': model.state_dict(),
                    'optimizer_state_dict': optimizer.state_dict(), 'train_loss': avg_train_loss,
                    'val_loss': avg_val_loss, 'metrics': metrics, 'user_mapping': user_mapping,
                    'item_mapping': item_mapping, 'config': config}
            if rank == 0:
                save_path.parent.mkdir(exist_ok=True, parents=True)
                torch.save(ckpt, save_path)
                print(f'\n New best model saved! Recall@10: {best_recall:.4f}')
        else:
            patience_counter += 1
            print(f'\n No improvement. Patience: {patience_counter}/{patience}')
            if patience_counter >= patience:
                print(f'\n Early stopping triggered after {epoch} epochs')
                break
        print(f"Current learning rate: {optimizer.param_groups[0]['lr']:.6f}")
    print(f"\n{'=' * 70}\nTraining completed!\nBest Recall@10: {best_recall:.4f}\n{'=' * 70}")
    return model, best_recall


def _cli():
    ap = argparse.ArgumentParser(description=__doc__.split('\n')[0])
    ap.add_argument('--config', default='config.yaml')
    ap.add_argument('--train', default='./data/cleaned/train_set.pkl')
    ap.add_argument('--val', default='./data/cleaned/val_set.pkl')
    ap.add_argument('--items', default='./data/cleaned/item_set.pkl')
    ap.add_argument('--metadata-config', default='metadata_config.yaml')
    ap.add_argument('--checkpoints', default='./checkpoints')
    ap.add_argument('--epochs', type=int, default=None)
    a = ap.parse_args()
    main(a.config, a.train, a.val, a.items, a.metadata_config, a.checkpoints, a.epochs)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == '__main__':
    _cli()
