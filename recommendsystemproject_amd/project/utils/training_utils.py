"""Training step and validation — drop-in for project/utils/training_utils.py
(to_device, train_one_epoch, extract_item_id, build_user_history, validate).

train_one_epoch runs the reference step body (training_utils.py:28-60; T15) on the HIP path:
zero_grad (one memset) -> forward -> compute_loss -> backward -> [RCCL all-reduce of the flat
gradient when torch.distributed is initialised] -> clip_grad_norm_(max_grad_norm) fused into
the Adam kernel -> scheduler. The per-step loss stays on the device (the reference's
loss.item() sync happens only at log points and at the end of the epoch).

validate (training_utils.py:121-275) keeps the reference's signature and result
({k: Recall@k}) but scores, masks, ranks and counts hits on the device (retrieval.hip): the
reference's per-user Python masking loop and its [B, num_items] score matrix per k become one
history CSR, per-chunk MFMA scores, a radix-select top-K and a hit-count kernel.
"""
import torch
from tqdm import tqdm

from recommendsystemproject_amd import dist as rdist
from recommendsystemproject_amd.optim import Adam, clip_grad_norm_


def to_device(data, device):
    """Recursively move tensors (dict / list nesting) to `device` (training_utils.py:5-16)."""
    if isinstance(data, torch.Tensor):
        return data.to(device, non_blocking=True)
    if isinstance(data, dict):
        return {k: to_device(v, device) for k, v in data.items()}
    if isinstance(data, list):
        return [to_device(v, device) for v in data]
    return data


def extract_item_id(item_batch, feature_name='movie_id_enc', feature_type='sparse', item_id_col=0):
    """training_utils.py:72-101 (T14: sparse column 0 regardless of the feature name)."""
    if feature_type == 'sparse':
        sparse_matrix = item_batch.get('sparse')
        if sparse_matrix is not None:
            return sparse_matrix[:, item_id_col]
    elif feature_type == 'dense':
        dense_matrix = item_batch.get('dense')
        if dense_matrix is not None:
            return dense_matrix[:, 0]
    elif feature_type == 'sequence':
        seq_dict = item_batch.get('sequence', {})
        if feature_name in seq_dict:
            return seq_dict[feature_name][:, 0]
    raise ValueError(f"Could not extract item ID '{feature_name}' from batch")


def build_user_history(train_df, user_col='user_id_enc', item_col='movie_id_enc'):
    """user -> set of interacted items (training_utils.py:103-119)."""
    user_history = {}
    for user_id, item_id in zip(train_df[user_col], train_df[item_col]):
        user_history.setdefault(user_id, set()).add(item_id)
    return user_history


_ONES = {}


def backward_seed(loss):
    """A persistent device 1.0 to seed loss.backward() with: autograd's implicit ones_like(loss) is
    a fill launch per step on the step's critical path."""
    key = (loss.device, loss.dtype)
    one = _ONES.get(key)
    if one is None:
        one = _ONES[key] = torch.ones((), device=loss.device, dtype=loss.dtype)
    return one


def train_step(model, batch_data, optimizer, max_grad_norm=1.0, temperature=0.1,
               item_id_feature='movie_id_enc', item_id_type='sparse'):
    """One training step on a device-resident batch; returns the loss as a device scalar."""
    optimizer.zero_grad()
    user_emb, pos_item_emb, hard_neg_emb = model(batch_data)
    ids = extract_item_id(batch_data['item_tower'], feature_name=item_id_feature, feature_type=item_id_type)
    loss = model.compute_loss(user_emb, pos_item_emb, hard_neg_emb=hard_neg_emb, item_ids=ids,
                              temperature=temperature)
    with rdist.overlap(model):  # data parallel: each tower's all-reduce starts in the backward
        loss.backward(backward_seed(loss))
    rdist.allreduce_gradients(model, optimizer)
    if isinstance(optimizer, Adam):
        optimizer.step(clip_max_norm=max_grad_norm if max_grad_norm > 0 else None)
    else:
        if max_grad_norm > 0:
            clip_grad_norm_(model.parameters(), max_grad_norm)
        optimizer.step()
    return loss.detach()


def _check_errors(model, optimizer=None):
    """Device error flags -> the reference's exceptions (one sync; see TwoTowerModel.check_errors)
    and the lazy-Adam step-constant overflow (optim.Adam.check_errors)."""
    m = getattr(model, 'module', model)
    if hasattr(m, 'check_errors'):
        m.check_errors()
    if optimizer is not None and hasattr(optimizer, 'check_errors'):
        optimizer.check_errors()


def train_one_epoch(model, loader, optimizer, device, scheduler=None, log_every_n_batches=100,
                    epoch=None, max_grad_norm=1.0, temperature=0.1, item_id_feature='movie_id_enc',
                    item_id_type='sparse'):
    """Same signature and return value (average loss) as training_utils.py:19-70."""
    model.train()
    losses = []
    pbar = tqdm(loader, desc=f'Training Epoch {epoch}')
    for batch_idx, batch_data in enumerate(pbar):
        batch_data = to_device(batch_data, device)
        loss = train_step(model, batch_data, optimizer, max_grad_norm, temperature, item_id_feature,
                          item_id_type)
        if scheduler is not None:
            scheduler.step()
        losses.append(loss)
        if batch_idx % log_every_n_batches == 0:
            pbar.set_postfix({'loss': f'{loss.item():.4f}', 'lr': f"{optimizer.param_groups[0]['lr']:.6f}"})
            # the reference raises at the failing op (IndexError at the lookup, GenericTower.py:
            # 184-196; RuntimeError on NaN embeddings, TwoTowerModel.py:88-91); the device flags
            # are read here, where loss.item() has already synchronised
            _check_errors(model, optimizer)
    total = float(torch.stack(losses).sum().item()) if losses else 0.0
    _check_errors(model, optimizer)
    avg_loss = total / max(len(loader), 1)
    print(f'Epoch {epoch} finished. Avg Loss: {avg_loss:.4f}')
    return avg_loss


# ============================================================================ validation
def _history_csr(user_history, all_item_ids_cpu, device):
    """user -> [catalog column indices] as device CSR (off [U+1] int64, idx int32), with the
    reference's filters: items <= max catalog id that are in the catalog (training_utils.py:
    238-252)."""
    import numpy as np
    ids = np.asarray(all_item_ids_cpu, dtype=np.int64)
    max_id = int(ids.max())
    id_to_index = np.full(max_id + 1, -1, dtype=np.int64)
    id_to_index[ids] = np.arange(len(ids))
    def _uid(u):  # the reference's build_user_history can key by column NAME (list columns)
        try:
            return int(u)
        except (TypeError, ValueError):
            return -1
    users = [_uid(u) for u in user_history.keys() if _uid(u) >= 0]
    U = (max(users) + 1) if users else 0
    counts = np.zeros(U + 1, dtype=np.int64)
    cols = []
    for u in range(U):
        items = user_history.get(u, user_history.get(np.int64(u), ()))
        valid = [int(i) for i in items if 0 <= int(i) <= max_id]
        c = id_to_index[valid] if valid else np.zeros(0, dtype=np.int64)
        c = c[c >= 0]
        counts[u + 1] = len(c)
        cols.append(c)
    off = np.cumsum(counts)
    idx = np.concatenate(cols).astype(np.int32) if cols and off[-1] > 0 else np.zeros(1, dtype=np.int32)
    return (torch.from_numpy(off).to(device), torch.from_numpy(idx).to(device), U)


def retrieval_topk(user_emb, all_item_embs, K, user_ids=None, history=None, chunk=65536):
    """Top-K catalog columns per user by dot-product score: per column chunk the MFMA GEMM
    (scores never leave HBM), the device history mask and the device top-K; chunks' candidates
    are merged by one more top-K over their values. Returns int32 [B, K], best first."""
    from recommendsystemproject_amd import _hip, ops
    U = user_emb.contiguous()
    items = all_item_embs.contiguous()
    for t in (U, items) + ((user_ids,) + tuple(history[:2]) if history is not None and user_ids is not None else ()):
        _hip.require_device(t)
    B, D = int(U.shape[0]), int(U.shape[1])
    N = int(items.shape[0])
    if K > N:
        raise ValueError(f'selected index k out of range (k={K}, items={N})')
    dev = U.device
    stream = torch.cuda.current_stream().cuda_stream
    chunks = [(c0, min(chunk, N - c0)) for c0 in range(0, N, chunk)]
    ks = [min(K, n) for _, n in chunks]
    C = sum(ks)
    cand_i = torch.empty(B, C, device=dev, dtype=torch.int32)
    cand_v = torch.empty(B, C, device=dev, dtype=torch.float32)
    S = torch.empty(B, min(chunk, N), device=dev, dtype=torch.float32)
    pos = 0
    for (c0, n), k in zip(chunks, ks):
        ops.gemm(U, items[c0:c0 + n], S, B, n, D, transA=0, transB=1, lda=D, ldb=D, ldc=n)
        if history is not None and user_ids is not None:
            off, idx, nu = history
            _hip.call('rs_mask_history', S.data_ptr(), n, B, c0, n, user_ids.data_ptr(), int(user_ids.stride(0)),
                      off.data_ptr(), idx.data_ptr(), nu, stream)
        _hip.call('rs_topk_rows', S.data_ptr(), n, B, n, k, None, 0, c0, cand_i.data_ptr() + 4 * pos,
                  cand_v.data_ptr() + 4 * pos, C, stream)
        pos += k
    if len(chunks) == 1:
        return cand_i
    out = torch.empty(B, K, device=dev, dtype=torch.int32)
    _hip.call('rs_topk_rows', cand_v.data_ptr(), C, B, C, K, cand_i.data_ptr(), C, 0, out.data_ptr(), None, K,
              stream)
    return out


def validate(model, loader, item_loader, device, epoch, k_list=[10, 20],
             item_id_feature='movie_id_enc', item_id_type='sparse', item_id_col_idx=0,
             meta_data_loader=None, user_id_col_idx=None, log_embeddings=True, user_history=None):
    """training_utils.py:121-275 on the device: item index through the item tower (eval mode),
    loss, MFMA scores U I_all^T, history mask, top-K and hit counts without host round trips
    per user (the reference loops over users in Python); one sync at the end."""
    from recommendsystemproject_amd import _hip
    model.eval()
    k_list = list(k_list)
    Kmax = max(k_list)
    print("Pre-computing all item embeddings for Validation...")
    embs, ids_l = [], []
    with torch.no_grad():
        for item_batch in tqdm(item_loader, desc="Indexing Items"):
            item_batch = to_device(item_batch, device)
            embs.append(model.get_item_embeddings(item_batch))
            ids_l.append(extract_item_id(item_batch, feature_name='movie_id_enc', feature_type='sparse',
                                         item_id_col=0))
        all_item_embs = torch.cat(embs, dim=0)
        all_item_ids = torch.cat(ids_l, dim=0).view(-1).long()
    history = None
    if user_history is not None:
        history = _history_csr(user_history, all_item_ids.cpu().numpy(), all_item_embs.device)
    if log_embeddings and epoch is not None:
        _log_embedding_stats(all_item_embs, epoch)
    meta_iter = iter(meta_data_loader) if meta_data_loader is not None else None
    dev = all_item_embs.device
    total_loss = torch.zeros((), device=dev)
    hits = torch.zeros(len(k_list), dtype=torch.int32, device=dev)
    ks = torch.tensor(k_list, dtype=torch.int32, device=dev)
    num_samples = 0
    n_batches = 0
    stream = torch.cuda.current_stream().cuda_stream
    with torch.no_grad():
        for batch_data in tqdm(loader, desc="Validating"):
            batch_data = to_device(batch_data, device)
            user_emb, pos_item_emb, hard_neg_emb = model(batch_data)
            item_batch = batch_data.get('item_tower', {})
            if not item_batch:
                raise ValueError("batch_data does not contain 'item_tower' key")
            if item_id_type == 'sparse' and 'sparse' in item_batch:
                targets = item_batch['sparse'][:, item_id_col_idx]
            elif item_id_type == 'dense' and 'dense' in item_batch:
                targets = item_batch['dense'][:, item_id_col_idx]
            elif item_id_type == 'sequence' and 'sequence' in item_batch:
                targets = item_batch['sequence'][item_id_feature][:, 0]
            else:
                raise ValueError(f"Cannot extract target item IDs from batch. item_batch keys: "
                                 f"{item_batch.keys()}, looking for type: {item_id_type}")
            loss = model.compute_loss(user_emb, pos_item_emb, hard_neg_emb=hard_neg_emb, item_ids=targets)
            total_loss += loss
            user_ids = None
            if user_history is not None:
                if meta_iter is not None:
                    user_ids = next(meta_iter)['user_tower']['sparse'][:, 0]
                    user_ids = user_ids.to(dev)
                elif user_id_col_idx is not None:
                    user_ids = batch_data.get('user_tower', {})['sparse'][:, user_id_col_idx]
                else:
                    raise ValueError("Either metadata_loader or user_id_col_idx required")
                user_ids = user_ids.long()
            topk = retrieval_topk(user_emb, all_item_embs, Kmax, user_ids, history)
            tg = targets.long()
            _hip.require_device(tg)
            _hip.call('rs_recall_hits', topk.data_ptr(), int(topk.shape[0]), Kmax, all_item_ids.data_ptr(),
                      tg.data_ptr(), int(tg.stride(0)), ks.data_ptr(), len(k_list), hits.data_ptr(), stream)
            num_samples += int(targets.shape[0])
            n_batches += 1
    avg_loss = total_loss.item() / max(len(loader), 1)
    _check_errors(model)
    h = hits.cpu().tolist()
    acc_dict = {k: h[i] / max(num_samples, 1) for i, k in enumerate(k_list)}
    print(f"\nValidation Result - Loss: {avg_loss:.4f}")
    for k, acc in acc_dict.items():
        print(f"Recall@{k}: {acc:.4f}")
    return avg_loss, acc_dict


def _log_embedding_stats(all_item_embs, epoch):
    """Item-embedding diagnostics (training_utils.py:277-325; logging only)."""
    emb_std = all_item_embs.std(dim=0).mean().item()
    emb_mean_norm = all_item_embs.mean(dim=0).norm().item()
    num_items = all_item_embs.shape[0]
    if num_items > 1000:
        sample = all_item_embs[torch.randperm(num_items, device=all_item_embs.device)[:1000]]
    else:
        sample = all_item_embs
    dists = torch.cdist(sample, sample)
    mask = ~torch.eye(dists.shape[0], dtype=torch.bool, device=dists.device)
    print(f"\n{'=' * 70}")
    print(f"Epoch {epoch} - Item Embedding Diagnostics:")
    print(f"{'=' * 70}")
    print(f"  Item Embedding Std:       {emb_std:.6f}")
    print(f"  Item Embedding Mean Norm: {emb_mean_norm:.6f}")
    print(f"  Avg Pairwise Distance:    {dists[mask].mean().item():.6f}")
    print(f"  Min Pairwise Distance:    {dists[mask].min().item():.6f}")
    print(f"  Max Pairwise Distance:    {dists[mask].max().item():.6f}")
    print(f"  Total Items:              {num_items}")
