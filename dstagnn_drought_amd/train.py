"""Training driver: the counterpart of train_DSTAGNN_my.py on MI355X.

    python -m dstagnn_drought_amd.train --config configurations/PEMS08_dstagnn.conf
    torchrun --nproc-per-node 8 -m dstagnn_drought_amd.train --config ...   (one rank per GPU)

Same configuration files, graph loading, model construction (make_model), loss
(SmoothL1), optimiser (Adam, the config's learning rate), epoch loop, validation,
best-epoch checkpoints ``myexperiments/{dataset}/{model}_{h}h{d}d{w}w_channel{c}_{lr}/
epoch_{e}.params`` in the reference's state_dict format, and final test loss
(train_DSTAGNN_my.py:30-191).  Where the reference runs on torch_xla, this runs one
process per GPU with torch.distributed over RCCL:

  * ``xm.optimizer_step`` (:148, :158) = mean all-reduce of the gradients over the ranks
    (dp.GradAllReducer, bucketed, cheb-mask grads as their support) + ``optimizer.step()``.
    The reference's double step per batch (quirk 14: the step at :148 re-applies the
    previous batch's gradients before ``zero_grad``) is kept by default
    (``double_step=True``; its gradients are already reduced, so no second collective).
  * data parallelism shards the training set (DistributedSampler order: rank r takes
    positions r, r+W, ... of the epoch permutation) instead of every replica training on
    the full set (quirk 15); validation / test batches are split across ranks and their
    per-batch losses all-reduced, so the reported mean over batches is the reference's.
  * batches are cut on the device (one index_select per batch from HBM-resident tensors)
    instead of DataLoader collation + MpDeviceLoader; the epoch permutation is drawn as
    torch's RandomSampler draws it (a seed from the global RNG, then randperm), so the
    first epoch visits samples in the reference's order.
  * the missing ``graph`` key of the PEMS03/07/08 configs (quirk 16: KeyError in the
    reference) defaults to 'AG'.
"""
import argparse
import configparser
import math
import os
import random
import time

import numpy as np
import torch
import torch.distributed as dist
import torch.nn as nn
import torch.utils.data

from . import data as data_io
from .dp import GradAllReducer, mask_support_of
from .model import make_model, set_direct_grads, set_dropout


def seed_torch(seed):
    """train_DSTAGNN_my.py:20-28."""
    random.seed(seed)
    os.environ['PYTHONHASHSEED'] = str(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)


def _world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


class DeviceBatches:
    """Mini-batches of HBM-resident (x, y) tensors.  shuffle: a fresh permutation per epoch
    drawn as torch's shuffled DataLoader draws it (same global-RNG consumption); with
    world > 1 rank r takes permutation positions r, r+W, ... (DistributedSampler order,
    padded by wrapping so every rank runs the same number of steps)."""

    def __init__(self, x, y, batch_size, shuffle, rank=0, world=1):
        self.x, self.y, self.bs, self.shuffle = x, y, int(batch_size), shuffle
        self.rank, self.world = rank, world

    def _order(self):
        n = self.x.shape[0]
        # the permutation (and every global-RNG draw) exactly as iterating the reference's
        # shuffled DataLoader would make it: one batch of a DataLoader over the positions
        perm = next(iter(torch.utils.data.DataLoader(torch.arange(n), batch_size=n, shuffle=self.shuffle)))
        if self.world > 1:
            per = -(-n // self.world)
            perm = torch.cat([perm, perm[:per * self.world - n]])[self.rank::self.world]
        return perm

    def __len__(self):
        n = -(-self.x.shape[0] // self.world) if self.world > 1 else self.x.shape[0]
        return -(-n // self.bs)

    def __iter__(self):
        perm = self._order().to(self.x.device)
        for i in range(0, perm.numel(), self.bs):
            idx = perm[i:i + self.bs]
            yield self.x.index_select(0, idx), self.y.index_select(0, idx)


def eval_batches(net, x, y, batch_size, criterion):
    """Mean over batches of the batch-mean loss (train_DSTAGNN_my.py:164-172), with the
    batches split round-robin over the ranks and the sums all-reduced."""
    rank, world = _world()
    iter(torch.utils.data.DataLoader(range(1)))  # the global-RNG draw a DataLoader iteration makes
    n = x.shape[0]
    starts = list(range(0, n, batch_size))
    tot = torch.zeros(2, dtype=torch.float64, device=x.device)
    with torch.no_grad():
        for b in starts[rank::world]:
            tot[0] += criterion(net(x[b:b + batch_size]), y[b:b + batch_size]).double()
            tot[1] += 1
    if world > 1:
        dist.all_reduce(tot)
    return float(tot[0] / max(1.0, float(tot[1])))


def compute_val_loss_mstgcn(net, val_loader, criterion, sw, epoch, limit=None):
    """lib/utils1.py:348-383: mean validation loss over the batches of `val_loader`
    (eval mode, no grad); `sw` (a SummaryWriter or None) gets 'validation_loss'."""
    net.train(False)
    with torch.no_grad():
        tmp = []
        for batch_index, (encoder_inputs, labels) in enumerate(val_loader):
            loss = criterion(net(encoder_inputs), labels)
            tmp.append(loss.item())
            if (limit is not None) and batch_index >= limit:
                break
        validation_loss = sum(tmp) / len(tmp)
        if sw is not None:
            sw.add_scalar('validation_loss', validation_loss, epoch)
    return validation_loss


def predict_and_save_results_mstgcn(net, data_loader, data_target_tensor, global_step, _mean, _std, params_path,
                                    type):
    """lib/utils1.py:441-510: predictions over `data_loader`, saved with the de-normalised
    inputs as ``output_epoch_{step}_{type}.npz`` (keys input, prediction,
    data_target_tensor); returns the per-horizon [MAE, RMSE, MAPE] list + the overall three."""
    from sklearn.metrics import mean_absolute_error, mean_squared_error
    net.train(False)
    with torch.no_grad():
        data_target_tensor = data_target_tensor.cpu().numpy()
        prediction, inputs = [], []
        for encoder_inputs, labels in data_loader:
            inputs.append(encoder_inputs[:, :, 0:1].cpu().numpy())
            prediction.append(net(encoder_inputs).detach().cpu().numpy())
        inputs = data_io.re_normalization(np.concatenate(inputs, 0), _mean, _std)
        prediction = np.concatenate(prediction, 0)
        np.savez(os.path.join(params_path, 'output_epoch_%s_%s' % (global_step, type)), input=inputs,
                 prediction=prediction, data_target_tensor=data_target_tensor)
        excel_list = []
        for i in range(prediction.shape[2]):
            assert data_target_tensor.shape[0] == prediction.shape[0]
            t, p = data_target_tensor[:, :, i], prediction[:, :, i]
            excel_list.extend([mean_absolute_error(t, p), mean_squared_error(t, p) ** 0.5,
                               data_io.masked_mape_np(t, p, 0)])
        t, p = data_target_tensor.reshape(-1, 1), prediction.reshape(-1, 1)
        excel_list.extend([mean_absolute_error(t, p), mean_squared_error(t, p) ** 0.5,
                           data_io.masked_mape_np(t, p, 0)])
    return excel_list


def build(config, device):
    """Graphs + model exactly as train_DSTAGNN_my.py:62-107 (model built on CPU, then moved)."""
    dc, tc = config['Data'], config['Training']
    N = int(dc['num_of_vertices'])
    if dc['dataset_name'] in ['PEMS04', 'PEMS08', 'PEMS07', 'PEMS03']:
        adj_mx = data_io.get_adjacency_matrix2(dc['adj_filename'], N, id_filename=dc.get('id_filename'))
    else:
        adj_mx = data_io.load_weighted_adjacency_matrix2(dc['adj_filename'], N)
    adj_TMD = data_io.load_weighted_adjacency_matrix(dc['stag_filename'], N)
    adj_pa = data_io.load_PA(dc['strg_filename'])
    adj_mx, adj_TMD, adj_pa = torch.FloatTensor(adj_mx), torch.FloatTensor(adj_TMD), torch.FloatTensor(adj_pa)
    adj_merge = adj_mx if tc.get('graph', 'AG') == 'G' else adj_TMD
    net = make_model('cpu', int(tc['in_channels']), int(tc['nb_block']), int(tc['in_channels']), int(tc['K']),
                     int(tc['nb_chev_filter']), int(tc['nb_time_filter']), 1, adj_merge, adj_pa, adj_TMD,
                     int(dc['num_for_predict']), int(dc['len_input']), N, int(tc['d_model']), int(tc['d_k']),
                     int(tc['d_k']), int(tc['n_heads']))
    return net.to(device)


def params_path_of(config, root='myexperiments'):
    """train_DSTAGNN_my.py:115-123."""
    tc = config['Training']
    folder_dir = '{}_{}h{}d{}w_channel{}_{}'.format(tc['model_name'], tc['num_of_hours'], tc['num_of_days'],
                                                    tc['num_of_weeks'], tc['in_channels'],
                                                    float(tc['learning_rate']))
    return os.path.join(root, config['Data']['dataset_name'], folder_dir)


class HipAdam(torch.optim.Optimizer):
    """torch.optim.Adam as train_DSTAGNN_my.py:126 builds it (betas (0.9, 0.999), eps 1e-8, no
    weight decay) with the whole update in ONE launch of the library's Adam kernel
    (``dstagnn::adam_step``, csrc/optim.hip) over every parameter that has a gradient — torch's
    fused Adam takes four ~43 us launches after ~0.2 ms of host-side grouping at PEMS08
    nb_block=4.  fp32 CUDA parameters only; state per parameter as torch's Adam
    (``step``, ``exp_avg``, ``exp_avg_sq``)."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps))
        # per group, after a step whose gradient-carrying parameters all shared one step count:
        # (params list, which params had a gradient, those params, their state dicts,
        # exp_avgs, exp_avg_sqs, step).  The per-parameter grouping below costs ~2 us per
        # Parameter in Python (~0.3 ms at nb_block=4, with the GPU idle); the cached path
        # gathers the gradients and launches while the same parameters carry gradients.
        self._plans = {}

    def load_state_dict(self, state_dict):
        """Accepts HipAdam's and torch.optim.Adam's state_dicts alike: torch keeps ``step`` as a
        (float) tensor, HipAdam as a Python int (a tensor step would key ``by_step`` below by
        identity: one launch per parameter and no cached plan), so it is converted here."""
        self._plans = {}
        super().load_state_dict(state_dict)
        for st in self.state.values():
            if "step" in st and torch.is_tensor(st["step"]):
                st["step"] = int(st["step"].item())

    def state_dict(self):
        """torch.optim.Adam's format: ``step`` as a float32 CPU tensor (the live state keeps the
        int; the returned per-parameter dicts are copies)."""
        sd = super().state_dict()
        sd["state"] = {k: (dict(v, step=torch.tensor(float(v["step"]), dtype=torch.float32))
                           if "step" in v and not torch.is_tensor(v["step"]) else v)
                       for k, v in sd["state"].items()}
        return sd

    def zero_grad(self, set_to_none=True):
        """torch's zero_grad(set_to_none=True) spends ~1 us per parameter in profiler /
        foreach bookkeeping (~0.15 ms at nb_block=4, before the forward can start); dropping
        the references is all it does here."""
        if not set_to_none:
            return super().zero_grad(set_to_none=False)
        for group in self.param_groups:
            for p in group["params"]:
                p.grad = None

    def _fast_step(self, ops, group):
        plan = self._plans.get(id(group))
        params = group["params"]
        if plan is None or plan[0] is not params or len(plan[1]) != len(params):
            return False
        grads = [p.grad for p in params]
        if [g is not None for g in grads] != plan[1]:
            return False
        _, present, ps, states, ms, vs, t = plan
        gs = [g for g in grads if g is not None]
        t += 1
        b1, b2 = group["betas"]
        ops.adam_step(ps, gs, ms, vs, b1, b2, group["eps"], group["lr"] / (1.0 - b1 ** t),
                      math.sqrt(1.0 - b2 ** t))
        for st in states:
            st["step"] = t
        self._plans[id(group)] = plan[:6] + (t,)
        return True

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        from . import _lib
        ops = _lib.load()
        for group in self.param_groups:
            if self._fast_step(ops, group):
                continue
            self._plans.pop(id(group), None)
            b1, b2 = group["betas"]
            lr, eps = group["lr"], group["eps"]
            by_step = {}
            for p in group["params"]:
                g = p.grad
                if g is None:
                    continue
                if g.is_sparse or not p.is_cuda or p.dtype != torch.float32:
                    raise RuntimeError("HipAdam: dense fp32 CUDA parameters only")
                st = self.state[p]
                if not st:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                st["step"] = int(st["step"]) + 1  # (a tensor step from a foreign state_dict)
                lists = by_step.setdefault(st["step"], ([], [], [], []))
                lists[0].append(p if p.is_contiguous() else p.data)
                lists[1].append(g)  # a strided gradient is copied contiguous by the op
                lists[2].append(st["exp_avg"])
                lists[3].append(st["exp_avg_sq"])
            for t, (ps, gs, ms, vs) in by_step.items():
                if any(not q.is_contiguous() for q in ps):
                    raise RuntimeError("HipAdam: non-contiguous parameter")
                step_size = lr / (1.0 - b1 ** t)
                bc2_sqrt = math.sqrt(1.0 - b2 ** t)
                ops.adam_step(ps, gs, ms, vs, b1, b2, eps, step_size, bc2_sqrt)
            if len(by_step) == 1:
                (t, (ps, _, ms, vs)), = by_step.items()
                present = [p.grad is not None for p in group["params"]]
                self._plans[id(group)] = (group["params"], present, ps, [self.state[p] for p in ps], ms, vs, t)
        return loss


def make_adam(params, lr):
    """The driver's optimiser (train_DSTAGNN_my.py:126): HipAdam (one launch) when every
    parameter is an fp32 GPU tensor; DSTAGNN_ADAM=torch-fused / torch for torch's fused or
    default Adam (A/B)."""
    params = list(params)
    mode = os.environ.get("DSTAGNN_ADAM", "hip")
    on_gpu = bool(params) and all(p.is_cuda and p.dtype == torch.float32 for p in params)
    if on_gpu and mode == "hip":
        return HipAdam(params, lr=lr)
    if on_gpu and mode == "torch-fused":
        return torch.optim.Adam(params, lr=lr, fused=True)
    return torch.optim.Adam(params, lr=lr)


def fit(net, train_x, train_y, val_x, val_y, *, epochs, start_epoch=0, batch_size, lr, params_path,
        double_step=True, max_batches=None, log=print):
    """The epoch loop of train_DSTAGNN_my.py:136-178.  Returns (best_epoch, best_val, history)."""
    rank, world = _world()
    criterion = nn.SmoothL1Loss().to(train_x.device)
    optimizer = make_adam(net.parameters(), lr)
    reducer = None
    if world > 1:  # block gradients all-reduced beside the backward (attach)
        reducer = GradAllReducer(net.named_parameters(), mask_support=mask_support_of(net)).attach(net)
    loader = DeviceBatches(train_x, train_y, batch_size, True, rank, world)

    def optimizer_step(reduce=True):  # xm.optimizer_step
        if reducer is not None and reduce:
            reducer.all_reduce()
        optimizer.step()

    best_val, best_epoch, history = float('inf'), 0, []
    for epoch in range(start_epoch, epochs):
        net.train()
        t0 = time.time()
        total = torch.zeros((), dtype=torch.float64, device=train_x.device)
        nb = 0
        for batch_idx, (encoder_inputs, labels) in enumerate(loader):
            if max_batches is not None and batch_idx >= max_batches:
                break
            if double_step:
                optimizer_step(reduce=False)  # :148 re-applies the (already reduced) previous grads
            optimizer.zero_grad()
            loss = criterion(net(encoder_inputs), labels)
            loss.backward()
            optimizer_step()
            total += loss.detach().double()
            nb += 1
        net.eval()
        val = eval_batches(net, val_x, val_y, batch_size, criterion)
        history.append({"epoch": epoch, "train_loss": float(total) / max(1, nb), "val_loss": val,
                        "time_s": time.time() - t0, "batches": nb})
        if rank == 0:
            log(f'Epoch {epoch} Val Loss: {val:.4f} Time: {time.time() - t0:.2f}s')
            if val < best_val:
                best_val, best_epoch = val, epoch
                torch.save({k: v.detach().cpu() for k, v in net.state_dict().items()},
                           os.path.join(params_path, f'epoch_{epoch}.params'))
        elif val < best_val:
            best_val, best_epoch = val, epoch
    return best_epoch, best_val, history


def load_best(net, path):
    """train_DSTAGNN_my.py:184 (torch.load of the best checkpoint).  Only rank 0 wrote the file
    and only rank 0 reads it; the other ranks receive its tensors by broadcast (no shared
    filesystem assumed)."""
    rank, world = _world()
    if rank == 0:
        net.load_state_dict(torch.load(path, weights_only=True))
    if world > 1:
        with torch.no_grad():
            for t in net.state_dict().values():
                dist.broadcast(t, src=0)


def run(config_path, *, epochs=None, double_step=True, dropout=None, max_batches=None, root='myexperiments',
        log=print):
    """Whole script: data, graphs, model, training, best-checkpoint test loss."""
    config = configparser.ConfigParser()
    config.read(config_path)
    dc, tc = config['Data'], config['Training']
    rank, world = _world()
    device = torch.device('cuda', torch.cuda.current_device()) if torch.cuda.is_available() else torch.device('cpu')
    seed_torch(1)
    (train_x, train_loader, train_y, val_x, _, val_y, test_x, _, test_y, mean, std) = \
        data_io.load_graphdata_channel1(dc['graph_signal_matrix_filename'], int(tc['num_of_hours']),
                                        int(tc['num_of_days']), int(tc['num_of_weeks']), 'cpu',
                                        int(tc['batch_size']))
    next(iter(train_loader))  # the reference probes one batch (:59-61): same RNG draw before the init
    net = build(config, device)
    set_direct_grads(net)  # the loop only uses loss.backward() + .grad
    if dropout is not None:
        set_dropout(net, dropout)
    train_x, train_y, val_x, val_y, test_x, test_y = (t.to(device) for t in
                                                      (train_x, train_y, val_x, val_y, test_x, test_y))
    params_path = params_path_of(config, root)
    if rank == 0:
        os.makedirs(params_path, exist_ok=True)
        log(f'Params path: {params_path}')
    bs = int(tc['batch_size'])
    n_epochs = int(tc['epochs']) if epochs is None else int(epochs)
    best_epoch, best_val, history = fit(net, train_x, train_y, val_x, val_y, epochs=n_epochs,
                                        start_epoch=int(tc['start_epoch']), batch_size=bs,
                                        lr=float(tc['learning_rate']), params_path=params_path,
                                        double_step=double_step, max_batches=max_batches, log=log)
    load_best(net, os.path.join(params_path, f'epoch_{best_epoch}.params'))
    net.eval()
    test_loss = eval_batches(net, test_x, test_y, bs, nn.SmoothL1Loss())
    if rank == 0:
        log(f'Final Test Loss: {test_loss:.4f}')
    return {"best_epoch": best_epoch, "best_val": best_val, "test_loss": test_loss, "history": history,
            "params_path": params_path, "net": net}


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--config", default='configurations/PEMS04_dstagnn.conf', type=str)
    ap.add_argument("--epochs", type=int, default=None, help="override [Training] epochs")
    ap.add_argument("--max-batches", type=int, default=None, help="cap the training batches per epoch")
    ap.add_argument("--no-double-step", action="store_true",
                    help="one optimizer step per batch (the reference steps twice: quirk 14)")
    ap.add_argument("--dropout", type=float, default=None, help="override the blocks' Dropout(0.05)")
    ap.add_argument("--out-root", default="myexperiments")
    a = ap.parse_args(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        local = int(os.environ.get("LOCAL_RANK", "0"))
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    try:
        run(a.config, epochs=a.epochs, double_step=not a.no_double_step, dropout=a.dropout,
            max_batches=a.max_batches, root=a.out_root)
    finally:
        if world > 1:
            dist.destroy_process_group()


if __name__ == "__main__":
    main()
