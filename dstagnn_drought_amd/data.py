"""Graph and data I/O of the DSTAGNN pipeline, host side.

Same names, arguments, file formats and outputs as the reference's
  * ``lib/dataloader.py:5-23``   load_weighted_adjacency_matrix / load_PA /
                                 load_weighted_adjacency_matrix2 (CSV graphs -> ndarray)
  * ``lib/utils1.py:92-145``     get_adjacency_matrix2 (edge-list CSV -> 0/1 adjacency)
  * ``lib/utils1.py:294-343``    load_graphdata_channel1 (``*_r{h}_d{d}_w{w}_dstagnn.npz``
                                 -> tensors + DataLoaders)
  * ``lib/utils1.py:17-19``      re_normalization
  * ``lib/metrics.py:6-16``      masked_mape_np
  * ``prepareData.py:5-161``     search_data / get_sample_indices /
                                 read_and_generate_dataset / normalization
so a user of the reference finds the same entry points.  The windowing is restated as one
vectorised gather over all label positions instead of the reference's per-index Python
loop (identical arrays, checked against files the reference itself wrote:
tests/golden/gen_golden_data.py), which matters at GAMBIA scale.  Everything here is
numpy / pandas / torch-CPU plumbing; the compute path is the HIP library.
"""
import csv
import os

import numpy as np
import pandas as pd
import torch
import torch.utils.data


# ---------------------------------------------------------------------------------------
# graph files (lib/dataloader.py, lib/utils1.py)
# ---------------------------------------------------------------------------------------
def load_weighted_adjacency_matrix(file_path, num_v):
    """Dense CSV (no header) -> float64 0/1 matrix of its positive entries (lib/dataloader.py:5-9).
    ``num_v`` is unused, as in the reference."""
    df = pd.read_csv(file_path, header=None).to_numpy()
    return np.float64(df > 0)


def load_PA(file_path):
    """STRG (``strg_*.csv``) -> float64 0/1 matrix (lib/dataloader.py:11-15)."""
    df = pd.read_csv(file_path, header=None).to_numpy()
    return np.float64(df > 0)


def load_weighted_adjacency_matrix2(file_path, num_v):
    """Dense CSV -> (A > 0) as int64 minus the identity, float64 (lib/dataloader.py:17-23)."""
    df = pd.read_csv(file_path, header=None).to_numpy()
    return np.int64(df > 0) - np.identity(num_v)


def get_adjacency_matrix2(distance_df_filename, num_of_vertices, type_='connectivity', id_filename=None):
    """Edge-list CSV ``from,to,cost`` (header skipped) -> float32 (N, N) (lib/utils1.py:92-145).

    Reference behaviour kept: with ``id_filename`` the ids are remapped and both directions
    are set; without it only ``A[i, j] = 1`` (directed) for 'connectivity'; any other
    ``type_`` raises ValueError (the reference's ``type == 'distance'`` branch compares the
    builtin ``type`` and is unreachable, so 'distance' raises too).  Rows with a field
    count other than 3 are skipped.
    """
    A = np.zeros((int(num_of_vertices), int(num_of_vertices)), dtype=np.float32)
    if id_filename:
        with open(id_filename, 'r') as f:
            id_dict = {int(i): idx for idx, i in enumerate(f.read().strip().split('\n'))}
        with open(distance_df_filename, 'r') as f:
            f.readline()
            for row in csv.reader(f):
                if len(row) != 3:
                    continue
                i, j = id_dict[int(row[0])], id_dict[int(row[1])]
                float(row[2])
                A[i, j] = 1
                A[j, i] = 1
        return A
    with open(distance_df_filename, 'r') as f:
        f.readline()
        for row in csv.reader(f):
            if len(row) != 3:
                continue
            i, j = int(row[0]), int(row[1])
            float(row[2])
            if type_ == 'connectivity':
                A[i, j] = 1
            else:
                raise ValueError("type_ error, must be connectivity or distance!")
    return A


# ---------------------------------------------------------------------------------------
# metrics / normalisation (lib/metrics.py, lib/utils1.py)
# ---------------------------------------------------------------------------------------
def masked_mape_np(y_true, y_pred, null_val=np.nan):
    """MAPE in percent over entries != null_val (NaN: non-NaN), lib/metrics.py:6-16."""
    with np.errstate(divide='ignore', invalid='ignore'):
        if np.isnan(null_val):
            mask = ~np.isnan(y_true)
        else:
            mask = np.not_equal(y_true, null_val)
        mask = mask.astype('float32')
        mask /= np.mean(mask)
        mape = np.abs(np.divide(np.subtract(y_pred, y_true).astype('float32'), y_true))
        mape = np.nan_to_num(mask * mape)
        return np.mean(mape) * 100


def re_normalization(x, mean, std):
    return x * std + mean


def normalization(train, val, test):
    """z-score with the training split's mean/std over axes (0, 1, 3), prepareData.py:149-161."""
    assert train.shape[1:] == val.shape[1:] and val.shape[1:] == test.shape[1:]
    mean = train.mean(axis=(0, 1, 3), keepdims=True)
    std = train.std(axis=(0, 1, 3), keepdims=True)
    return {'_mean': mean, '_std': std}, (train - mean) / std, (val - mean) / std, (test - mean) / std


# ---------------------------------------------------------------------------------------
# windowing (prepareData.py)
# ---------------------------------------------------------------------------------------
def search_data(sequence_length, num_of_depend, label_start_idx, num_for_predict, units, points_per_hour):
    """Input windows [(start, end)] of one dependency kind, oldest first, or None
    (prepareData.py:5-24)."""
    if points_per_hour < 0:
        raise ValueError("points_per_hour should be greater than 0!")
    if label_start_idx + num_for_predict > sequence_length:
        return None
    x_idx = []
    for i in range(1, num_of_depend + 1):
        start_idx = label_start_idx - points_per_hour * units * i
        if start_idx < 0:
            return None
        x_idx.append((start_idx, start_idx + num_for_predict))
    return x_idx[::-1]


def get_sample_indices(data_sequence, num_of_weeks, num_of_days, num_of_hours, label_start_idx, num_for_predict,
                       points_per_hour=1):
    """(week, day, hour, target) samples of one label position (prepareData.py:26-61)."""
    if label_start_idx + num_for_predict > data_sequence.shape[0]:
        return None, None, None, None
    out = []
    for depend, units in ((num_of_weeks, 7 * 24), (num_of_days, 24), (num_of_hours, 1)):
        if depend > 0:
            idx = search_data(data_sequence.shape[0], depend, label_start_idx, num_for_predict, units,
                              points_per_hour)
            if not idx:
                return None, None, None, None
            out.append(np.concatenate([data_sequence[i:j] for i, j in idx], axis=0))
        else:
            out.append(None)
    target = data_sequence[label_start_idx: label_start_idx + num_for_predict]
    return out[0], out[1], out[2], target


def _valid_labels(T, num_of_weeks, num_of_days, num_of_hours, num_for_predict, points_per_hour):
    """Label positions read_and_generate_dataset keeps: the target fits and every enabled
    dependency kind has all its windows at start >= 0 (prepareData.py:71-80)."""
    comps = [(d, u) for d, u in ((num_of_weeks, 7 * 24), (num_of_days, 24), (num_of_hours, 1)) if d > 0]
    if not comps or points_per_hour < 0:
        if points_per_hour < 0 and comps:
            raise ValueError("points_per_hour should be greater than 0!")
        return np.zeros(0, dtype=np.int64), comps
    lo = max(points_per_hour * u * d for d, u in comps)
    return np.arange(lo, T - num_for_predict + 1, dtype=np.int64), comps


def read_and_generate_dataset(graph_signal_matrix_filename, num_of_weeks, num_of_days, num_of_hours,
                              num_for_predict, points_per_hour=1, save=False):
    """``data`` (T, N, F) of an .npz -> train/val/test windows (60/20/20 split by label
    position), z-normalised with the training statistics; optionally saved as
    ``{file}_r{h}_d{d}_w{w}_dstagnn.npz`` beside the input (prepareData.py:63-147).

    x (S, N, F, Tin): the enabled dependency kinds (week, day, hour) concatenated on the
    last axis, each its windows oldest first; target (S, N, num_for_predict) = the LAST
    feature over the predicted steps; timestamp (S, 1) = the label position.
    """
    data_seq = np.load(graph_signal_matrix_filename)['data']
    if data_seq.ndim == 4:
        data_seq = data_seq.squeeze(axis=2)
    T = data_seq.shape[0]
    labels, comps = _valid_labels(T, num_of_weeks, num_of_days, num_of_hours, num_for_predict, points_per_hour)
    # window starts per label: for each kind, i = depend .. 1 (oldest first), then + arange(nfp)
    starts = [labels[:, None] - points_per_hour * u * np.arange(d, 0, -1)[None, :] for d, u in comps]
    tsteps = (np.concatenate(starts, axis=1)[:, :, None] + np.arange(num_for_predict)[None, None, :]).reshape(
        len(labels), -1) if comps else np.zeros((0, 0), dtype=np.int64)
    # gather (S, Tin, N, F) -> (S, N, F, Tin)
    # kept as the (S, Tin, N, F)-ordered view: the reference's np.concatenate result has that
    # same memory order, so the normalisation's float reductions run in the same order
    # (bit-identical statistics)
    x_all = data_seq[tsteps].transpose(0, 2, 3, 1) if len(labels) else None
    tgt_steps = labels[:, None] + np.arange(num_for_predict)[None, :]
    y_all = np.ascontiguousarray(data_seq[tgt_steps][..., -1].transpose(0, 2, 1)) if len(labels) else None
    ts_all = labels[:, None]

    S = len(labels)
    s1, s2 = int(S * 0.6), int(S * 0.8)
    if x_all is None or s1 == 0 or s2 == s1 or S == s2:
        raise ValueError("need at least one sample in each of the train / val / test splits "
                         "(the reference fails in np.concatenate)")
    train_x, val_x, test_x = x_all[:s1], x_all[s1:s2], x_all[s2:]
    stats, train_x_norm, val_x_norm, test_x_norm = normalization(train_x, val_x, test_x)
    all_data = {
        'train': {'x': train_x_norm, 'target': y_all[:s1], 'timestamp': ts_all[:s1]},
        'val': {'x': val_x_norm, 'target': y_all[s1:s2], 'timestamp': ts_all[s1:s2]},
        'test': {'x': test_x_norm, 'target': y_all[s2:], 'timestamp': ts_all[s2:]},
        'stats': {'_mean': stats['_mean'], '_std': stats['_std']},
    }
    if save:
        np.savez_compressed(dataset_filename(graph_signal_matrix_filename, num_of_hours, num_of_days, num_of_weeks),
                            train_x=all_data['train']['x'], train_target=all_data['train']['target'],
                            train_timestamp=all_data['train']['timestamp'],
                            val_x=all_data['val']['x'], val_target=all_data['val']['target'],
                            val_timestamp=all_data['val']['timestamp'],
                            test_x=all_data['test']['x'], test_target=all_data['test']['target'],
                            test_timestamp=all_data['test']['timestamp'],
                            mean=all_data['stats']['_mean'], std=all_data['stats']['_std'])
    return all_data


def dataset_filename(graph_signal_matrix_filename, num_of_hours, num_of_days, num_of_weeks):
    """``{dir}/{stem}_r{h}_d{d}_w{w}_dstagnn`` (prepareData.py:132-134, lib/utils1.py:295-297)."""
    file = os.path.basename(graph_signal_matrix_filename).split('.')[0]
    dirpath = os.path.dirname(graph_signal_matrix_filename)
    return os.path.join(dirpath, f"{file}_r{num_of_hours}_d{num_of_days}_w{num_of_weeks}") + '_dstagnn'


# ---------------------------------------------------------------------------------------
# training data (lib/utils1.py:294-343)
# ---------------------------------------------------------------------------------------
def load_graphdata_channel1(graph_signal_matrix_filename, num_of_hours, num_of_days, num_of_weeks, DEVICE,
                            batch_size, shuffle=True, sampler=None):
    """The prepared ``*_dstagnn.npz`` -> (train_x, train_loader, train_target, val_x, val_loader,
    val_target, test_x, test_loader, test_target, mean, std), float32 tensors on DEVICE,
    TensorDataset loaders (train shuffled).  ``sampler`` (optional, e.g. a
    DistributedSampler factory ``f(dataset) -> Sampler``) shards the training set for
    data-parallel runs; it replaces shuffle, as torch's DataLoader requires."""
    filename = dataset_filename(graph_signal_matrix_filename, num_of_hours, num_of_days, num_of_weeks)
    print('load file:', filename)
    file_data = np.load(filename + '.npz')
    t = {}
    for split in ('train', 'val', 'test'):
        t[split + '_x'] = torch.from_numpy(file_data[split + '_x']).type(torch.FloatTensor).to(DEVICE)
        t[split + '_target'] = torch.from_numpy(file_data[split + '_target']).type(torch.FloatTensor).to(DEVICE)
    mean, std = file_data['mean'], file_data['std']
    train_ds = torch.utils.data.TensorDataset(t['train_x'], t['train_target'])
    if sampler is not None:
        train_loader = torch.utils.data.DataLoader(train_ds, batch_size=batch_size, sampler=sampler(train_ds))
    else:
        train_loader = torch.utils.data.DataLoader(train_ds, batch_size=batch_size, shuffle=shuffle)
    val_loader = torch.utils.data.DataLoader(torch.utils.data.TensorDataset(t['val_x'], t['val_target']),
                                             batch_size=batch_size, shuffle=False)
    test_loader = torch.utils.data.DataLoader(torch.utils.data.TensorDataset(t['test_x'], t['test_target']),
                                              batch_size=batch_size, shuffle=False)
    print('train:', t['train_x'].size(), t['train_target'].size())
    print('val:', t['val_x'].size(), t['val_target'].size())
    print('test:', t['test_x'].size(), t['test_target'].size())
    return (t['train_x'], train_loader, t['train_target'], t['val_x'], val_loader, t['val_target'],
            t['test_x'], test_loader, t['test_target'], mean, std)


def main(argv=None):
    """``python -m dstagnn_drought_amd.data --config X.conf``: prepareData.py's CLI
    (prepareData.py:164-192) — window the config's series and save the ``*_dstagnn.npz``."""
    import argparse
    import configparser
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default='configurations/GAMBIA_dstagnn.conf', type=str)
    a = ap.parse_args(argv)
    config = configparser.ConfigParser()
    config.read(a.config)
    dc, tc = config['Data'], config['Training']
    return read_and_generate_dataset(dc['graph_signal_matrix_filename'], int(tc['num_of_weeks']),
                                     int(tc['num_of_days']), int(tc['num_of_hours']), int(dc['num_for_predict']),
                                     points_per_hour=int(dc['points_per_hour']), save=True)


if __name__ == "__main__":
    main()
