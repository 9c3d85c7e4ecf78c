"""TwoTowerModel — drop-in for project/models/TwoTower/TwoTowerModel.py (same API:
forward / predict / get_item_embeddings / compute_loss / set_feature_mappings). compute_loss is
one custom op, rsys::inbatch_softmax_loss (library.py; kernels in functions.InBatchLossFn): U I^T
on the MFMA, collision mask, hard negatives and the softmax cross-entropy fused."""
import os

import torch
import torch.nn as nn

from recommendsystemproject_amd import _hip, library, streams
from recommendsystemproject_amd import dist as rdist
from recommendsystemproject_amd.flat import ensure_flat


class TwoTowerModel(nn.Module):
    def __init__(self, user_tower, item_tower, user_feature_mapping=None, item_feature_mapping=None):
        super().__init__()
        self.user_tower = user_tower
        self.item_tower = item_tower
        self.user_feature_mapping = user_feature_mapping
        self.item_feature_mapping = item_feature_mapping
        # the reference raises on NaN embeddings with a host sync per step (TwoTowerModel.py:88-91).
        # Here every step ORs a device flag (rs_nan_check, no sync) and check_errors() raises the
        # same RuntimeError at the caller's next sync (train_one_epoch's log points, validate);
        # RSYS_CHECK_NAN=1 / model.check_nan = True restores the reference's per-step sync.
        self.check_nan = os.environ.get('RSYS_CHECK_NAN', '0') == '1'
        self.register_buffer('nan_flag', torch.zeros(1, dtype=torch.int32), persistent=False)

    def set_feature_mappings(self, user_mapping, item_mapping):
        self.user_feature_mapping = user_mapping
        self.item_feature_mapping = item_mapping

    def _side_stream(self, dev):
        """The item tower's stream: the two towers are independent until the loss, so the item
        tower (all small, latency-bound kernels at B = 4096) runs beside the user tower's encoder.
        RSYS_TOWER_STREAMS=0 keeps everything on the current stream."""
        if os.environ.get('RSYS_TOWER_STREAMS', '1') == '0':
            return None
        s = getattr(self, '_rs_side_stream', None)
        if s is None or s.device != dev:
            s = streams.side_stream(dev)
            self._rs_side_stream = s
        return s

    def _user_stream(self, dev):
        """RSYS_USER_STREAM=1 (or 'high': the highest stream priority): the user tower on a stream of
        its own instead of the current one -- the current stream then only forks the two towers
        and joins them before the loss. Off by default (measured no faster: DESIGN.md §5)."""
        mode = os.environ.get('RSYS_USER_STREAM', '0')
        if mode not in ('1', 'high'):
            return None
        s = getattr(self, '_rs_user_stream', None)
        if s is None or s.device != dev or getattr(self, '_rs_user_stream_mode', None) != mode:
            if mode == 'high':
                _, hi = torch.cuda.Stream.priority_range()
                s = streams.side_stream(dev, priority=hi)
            else:
                s = streams.side_stream(dev)
            self._rs_user_stream, self._rs_user_stream_mode = s, mode
        return s

    def forward(self, batch_data):
        """-> (user_emb [B,D], item_emb [B,D], hard_neg_emb [B,N,D] or None) (TwoTowerModel.py:35-62;
        T13: one item-tower pass per hard-negative slot, so BatchNorm statistics are per slot)."""
        try:
            return self._forward(batch_data)
        finally:
            rdist.end_forward()  # the batch agreement is this forward's only (dist.end_forward)

    def _forward(self, batch_data):
        dev = self.user_tower.feature_bn.weight.device
        _hip.require_device(self.user_tower.feature_bn.weight)
        ensure_flat(self)
        if rdist.is_active():
            # one gradient bucket per tower, all-reduced inside the backward (dist.overlap)
            rdist.setup_buckets(self, [self.user_tower, self.item_tower])
            # the batch's shapes over the ranks, in one all-reduce: the large tables' lookup calls
            # take their common shapes from it (no collective per call)
            rdist.agree_batch(batch_data)
        side = self._side_stream(dev)
        if side is not None and not streams.can_fork():
            side = None  # called on a side stream already: no fork of a fork (streams.py)
        if side is None or library.is_fake(self.user_tower.feature_bn.weight) or library.fake_mode_active():
            user_emb = self.user_tower(batch_data['user_tower'], self.user_feature_mapping)
            item_emb, hard_neg_emb = self._item_side(batch_data)
            return user_emb, item_emb, hard_neg_emb
        # fork: the item tower (and its hard-negative pass) on the side stream, the user tower on
        # the current one; join before the loss. Autograd runs each tower's backward on the stream
        # its forward used, so the backward overlaps the same way. (Round 5 measured the user
        # tower's smaller lookup chains forked onto the side stream ahead of the item tower
        # slower: C3 fp32 0.78 -> 0.82, C2 1.33 -> 1.35 ms per step.)
        main = torch.cuda.current_stream(dev)
        streams.set_root(main)  # collectives issued on the side streams run here (streams.on_root)
        side.wait_stream(main)
        ustream = self._user_stream(dev)
        # (round 6 measured the item tower created after the user tower -- its backward then issued
        # first, beside the user tower's -- slower: C2 1.244 -> 1.251-1.266, C3 fp32 0.711 -> 0.723)
        with torch.cuda.stream(side):
            item_emb, hard_neg_emb = self._item_side(batch_data)
        if ustream is not None:
            ustream.wait_stream(main)
            with torch.cuda.stream(ustream):
                user_emb = self.user_tower(batch_data['user_tower'], self.user_feature_mapping)
            main.wait_stream(ustream)
            user_emb.record_stream(main)
        else:
            user_emb = self.user_tower(batch_data['user_tower'], self.user_feature_mapping)
        main.wait_stream(side)
        outs = [t for t in (item_emb, hard_neg_emb) if t is not None]
        for t in outs:
            t.record_stream(main)  # made on the side stream, read by the loss on the main one
        if torch.is_grad_enabled() and item_emb.requires_grad:
            self._join_backward(main, [(side, outs)] + ([(ustream, [user_emb])] if ustream is not None else []))
        return user_emb, item_emb, hard_neg_emb

    @staticmethod
    def _join_backward(main, branches):
        """The loss's gradient (main stream) is read by each tower's backward on its own stream; the
        backward kernels write the flat gradient directly (no AccumulateGrad to synchronise on),
        so once per backward the main stream waits for every branch stream's last kernels.
        The hooks hold the streams only: a hook holding the tensor it is registered on is a
        cycle through the autograd graph that Python's collector cannot see, and it kept every
        step's graph -- and through its parameter edges the model and its flat buffers -- alive."""
        joined = []
        streams = [st for st, _ in branches]

        def hook_for(st):
            def _to(g):
                g.record_stream(st)
                if not joined:
                    joined.append(True)

                    def _join():
                        for s in streams:
                            main.wait_stream(s)
                    torch.autograd.Variable._execution_engine.queue_callback(_join)
                return g
            return _to

        for st, ts in branches:
            for t in ts:
                if t.requires_grad:
                    t.register_hook(hook_for(st))

    def _item_side(self, batch_data):
        item_emb = self.item_tower(batch_data['item_tower'], self.item_feature_mapping)
        hard_neg_emb = None
        negs = batch_data.get('hard_negatives') if isinstance(batch_data, dict) else None
        if negs:
            stacked = getattr(negs, 'stacked', None)
            if stacked is not None:
                # materialised by ItemCatalog: the N slots are already one [N*B] batch; one item-tower
                # pass with per-slot BatchNorm statistics == N separate passes (T13)
                N = len(negs)
                out = self.item_tower(stacked, self.item_feature_mapping, groups=N)
                B = out.shape[0] // N
                hard_neg_emb = out.view(N, B, out.shape[1]).transpose(0, 1)  # [B, N, D] view
            else:
                hard_neg_emb = torch.stack([self.item_tower(neg, self.item_feature_mapping)
                                            for neg in negs], dim=1)
        return item_emb, hard_neg_emb

    def predict(self, batch_data):
        user_emb, item_emb, _ = self.forward(batch_data)
        return (user_emb * item_emb).sum(dim=1)

    def get_item_embeddings(self, item_inputs):
        return self.item_tower(item_inputs, self.item_feature_mapping)

    _NAN_MSG = {1: 'Found NaN in User Embedding', 2: 'Found NaN in Item Embedding',
                4: 'Found NaN in Hard Negative Embedding'}

    def _flag_nan(self, pairs):
        """One rs_nan_check_many launch over [(tensor, bit)] (the loss inputs)."""
        import ctypes as C
        ts, bits = [], []
        for t, bit in pairs:
            if t.is_cuda and not t.is_contiguous() and t.dim() == 3 and t.transpose(0, 1).is_contiguous():
                t = t.transpose(0, 1)  # the grouped hard-negative pass's [B, N, D] view of [N, B, D]
            if not t.is_cuda or not t.is_contiguous() or t.data_ptr() % 16:
                t = t.contiguous()
            ts.append(t)
            bits.append(bit)
        if self.nan_flag.device != ts[0].device:
            self.nan_flag = self.nan_flag.to(ts[0].device)
        k = len(ts)
        xs = (C.c_void_p * k)(*[t.data_ptr() for t in ts])
        ns = (C.c_int64 * k)(*[t.numel() for t in ts])
        bs = (C.c_int * k)(*bits)
        _hip.call('rs_nan_check_many', k, C.addressof(xs), C.addressof(ns), C.addressof(bs),
                  self.nan_flag.data_ptr(), torch.cuda.current_stream(ts[0].device).cuda_stream)

    def check_errors(self):
        """Raise what the reference would have raised since the last check: RuntimeError for NaN
        loss inputs (TwoTowerModel.py:88-91, 99-100), IndexError for an embedding id outside its
        table (GenericTower.py:184-196). One host sync; call it where the host syncs anyway."""
        v = int(self.nan_flag.item())
        if v:
            self.nan_flag.zero_()
            for bit in (1, 2, 4):
                if v & bit:
                    raise RuntimeError(self._NAN_MSG[bit])
        for tower in (self.user_tower, self.item_tower):
            if hasattr(tower, 'check_errors'):
                tower.check_errors()

    @torch.no_grad()
    def compute_logits(self, user_emb, item_emb, item_ids=None, hard_neg_emb=None, temperature=0.1):
        """The logits compute_loss feeds to cross_entropy (TwoTowerModel.py:95-136): U I^T / T with
        off-diagonal equal-id collisions at -1e9, hard-negative logits appended, [B, B + N].
        compute_loss never materialises them; this builds them with the same HIP kernels (S on
        the f32 MFMA GEMM, rs_inbatch_logits) for diagnostics and parity checks."""
        from recommendsystemproject_amd import ops
        U, I = user_emb.contiguous(), item_emb.contiguous()
        B, D = int(U.shape[0]), int(U.shape[1])
        S = torch.empty(B, B, device=U.device, dtype=torch.float32)
        ops.gemm(U, I, S, B, B, D, transA=0, transB=1, lda=D, ldb=D, ldc=B)
        N, Hc, hsr, hss = 0, None, 0, 0
        if hard_neg_emb is not None:
            Hc = hard_neg_emb if hard_neg_emb.stride(2) == 1 else hard_neg_emb.contiguous()
            N, hsr, hss = int(Hc.shape[1]), int(Hc.stride(0)), int(Hc.stride(1))
        ids, st = None, 0
        if item_ids is not None:
            ids = item_ids.reshape(-1)
            ids = ids if ids.dtype == torch.int64 else ids.long()
            st = int(ids.stride(0))
        out = torch.empty(B, B + N, device=U.device, dtype=torch.float32)
        _hip.call('rs_inbatch_logits', S.data_ptr(), B, U.data_ptr(), ops.P(Hc), hsr, hss, ops.P(ids), st,
                  B, N, D, float(temperature), out.data_ptr(), B + N, ops.stream())
        return out

    def compute_loss(self, user_emb, item_emb, item_ids=None, hard_neg_emb=None, temperature=0.1):
        """In-batch softmax loss (TwoTowerModel.py:81-150)."""
        if not self.check_nan and user_emb.is_cuda and not library.is_fake(user_emb):
            self._flag_nan([(user_emb.detach(), 1), (item_emb.detach(), 2)] +
                           ([(hard_neg_emb.detach(), 4)] if hard_neg_emb is not None else []))
        if self.check_nan:
            if torch.isnan(user_emb).any():
                raise RuntimeError('Found NaN in User Embedding')
            if torch.isnan(item_emb).any():
                raise RuntimeError('Found NaN in Item Embedding')
        batch_size = user_emb.shape[0]
        if hard_neg_emb is not None:
            if self.check_nan and torch.isnan(hard_neg_emb).any():
                raise RuntimeError('Found NaN in Hard Negative Embedding')
            assert hard_neg_emb.dim() == 3, f'Expected shape [B, N, D], got {hard_neg_emb.shape}'
            assert hard_neg_emb.size(0) == batch_size, 'Batch size mismatch'
        return library.inbatch_softmax_loss(user_emb, item_emb, item_ids, hard_neg_emb, float(temperature))
