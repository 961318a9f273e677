"""Data utilities — drop-in for the reference's `util.py` (kimerein/tensor_regression), plus the
MI355X-native windowed view the gfx950 kernels read without materialising windows.

Reference surface kept (util.py:15-114): `set_device`, `squeeze_integers`, `WindowedDataset`,
`make_WindowedDataloader` (torch Dataset / DataLoader over an untiled (T, ...) series; sample
`idx` is the window `X[idx + win_range[0] : idx + win_range[1]]` with target `y[idx]`).

New: `windowed_view(X_untiled, y, win_range)` returns the SAME samples the dataset yields for
`idx` in `dataset.usable_idx`, as an overlapping strided tensor view
(N_windows, win_len, *feature_dims) with stride (F, F, ...) along the window axis — no copy, so
X stays T x F in HBM instead of N x win_len x F.  The fit/predict entry points accept such views
(`tr_plan_set_x_stride`): every kernel reads sample n at X + n*F.
"""
import copy

import numpy as np
import torch
from torch.utils.data import DataLoader, Dataset

__all__ = ["set_device", "squeeze_integers", "WindowedDataset", "make_WindowedDataloader", "windowed_view",
           "HostStream"]


def set_device(use_GPU=True, verbose=True):
    """'cuda' if a HIP device is available and requested, else 'cpu' (util.py:15-35)."""
    if use_GPU:
        device = "cuda" if torch.cuda.is_available() else "cpu"
        if device != "cuda":
            print("no GPU available. Using CPU.") if verbose else None
        else:
            print(f"device: '{device}'") if verbose else None
    else:
        device = "cpu"
        print(f"device: '{device}'") if verbose else None
    return device


def squeeze_integers(arr):
    """The reference's gap-closing loop, as is (util.py:37-61): for each value in [0, max] missing
    from the ORIGINAL array, every entry above it moves down by one while the loop runs, so
    [0,2,2,5] -> [0,1,1,3] and [7,2,7,4,1] -> [5,1,5,3,0] (the reference's docstring claims
    [3,2,3,1,0]; its code returns this)."""
    uniques = np.unique(arr)
    arr_squeezed = copy.deepcopy(arr)
    for val in np.arange(0, np.max(arr) + 1):
        if np.isin(val, uniques):
            continue
        arr_squeezed[arr_squeezed > val] = arr_squeezed[arr_squeezed > val] - 1
    return arr_squeezed


class WindowedDataset(Dataset):
    """Windows of an untiled series (util.py:67-98): item idx = (X[idx+w0 : idx+w1], y[idx])."""

    def __init__(self, X_untiled, y_input, win_range, transform=None, target_transform=None):
        self.X_untiled = X_untiled
        self.y_input = y_input
        self.win_range = win_range
        self.n_samples = y_input.shape[0]
        self.usable_idx = torch.arange(-self.win_range[0], self.n_samples - self.win_range[1] + 1)
        if X_untiled.shape[0] != y_input.shape[0]:
            raise ValueError('RH: X and y must have same first dimension shape')

    def __len__(self):
        return self.n_samples

    def check_bound_errors(self, idx):
        idx_toRemove = []
        for val in idx:
            if (val + self.win_range[0] < 0) or (val + self.win_range[1] > self.n_samples):
                idx_toRemove.append(val)
        if len(idx_toRemove) > 0:
            raise ValueError(f'RH: input idx is too close to edges. Remove idx: {idx_toRemove}')

    def __getitem__(self, idx):
        X_subset_tiled = self.X_untiled[idx + self.win_range[0]: idx + self.win_range[1]]
        y_subset = self.y_input[idx]
        return X_subset_tiled, y_subset


def make_WindowedDataloader(X, y, win_range=[-10, 10], batch_size=64, drop_last=True, **kwargs_dataloader):
    """Random-order minibatches of windows (util.py:100-114)."""
    dataset = WindowedDataset(X, y, win_range)
    sampler = torch.utils.data.SubsetRandomSampler(dataset.usable_idx, generator=None)
    if kwargs_dataloader is None:
        kwargs_dataloader = {'shuffle': False, 'pin_memory': False, 'num_workers': 0}
    dataloader = DataLoader(dataset, batch_size=batch_size, drop_last=drop_last, sampler=sampler,
                            **kwargs_dataloader)
    dataloader.sample_shape = [dataloader.batch_size] + list(dataset[-win_range[0]][0].shape)
    return dataloader, dataset, sampler


def windowed_view(X_untiled, y, win_range):
    """All windows of WindowedDataset(X_untiled, y, win_range) over `usable_idx`, in order, as a
    zero-copy strided view: returns (Xw, yw) with Xw[n] == X_untiled[n : n + win_len] (the window
    of idx = n - win_range[0]) and yw[n] == y[n - win_range[0]].

    X_untiled must be contiguous (T, *F); Xw has shape (T - win_len + 1, win_len, *F) and
    stride (F, F, *F-strides), i.e. consecutive samples overlap by win_len - 1 rows.
    """
    X_untiled = torch.as_tensor(X_untiled)
    if not X_untiled.is_contiguous():
        X_untiled = X_untiled.contiguous()
    w0, w1 = int(win_range[0]), int(win_range[1])
    L = w1 - w0
    T = X_untiled.shape[0]
    n = T - L + 1
    if L < 1 or n < 1:
        raise ValueError(f"window {win_range} does not fit a series of length {T}")
    feat = tuple(X_untiled.shape[1:])
    F = int(np.prod(feat)) if feat else 1
    inner = tuple(X_untiled.stride()[1:])
    Xw = X_untiled.as_strided((n, L) + feat, (F, F) + inner)
    y = torch.as_tensor(y)
    yw = y[-w0: -w0 + n]
    return Xw, yw


class HostStream:
    """A sample-major X that stays in (pinned) host memory and is streamed through two device
    buffers in chunks of `chunk_rows` samples every iteration — the out-of-core path for an X
    larger than the HBM one wants to spend.  Host→device copies run on
    their own HIP stream, double-buffered against the loss/gradient kernels of the previous
    chunk; the per-chunk gradient arenas are summed exactly like the shards of a multi-GPU fit."""

    def __init__(self, X, chunk_rows, device="cuda"):
        X = torch.as_tensor(X)
        if X.dtype != torch.float32:
            raise TypeError(f"the gfx950 path computes in fp32; got X of dtype {X.dtype}")
        if X.device.type != "cpu":
            raise ValueError("HostStream wraps a host (CPU) tensor")
        X = X.contiguous()
        self.X = X if X.is_pinned() else X.pin_memory()
        self.chunk_rows = max(1, int(chunk_rows))
        self.shape = tuple(X.shape)
        self.device = torch.device(device)
        self.dev_index = self.device.index if self.device.index is not None else torch.cuda.current_device()
        rows = min(self.chunk_rows, X.shape[0])
        self.bufs = [torch.empty((rows,) + tuple(X.shape[1:]), dtype=torch.float32, device=f"cuda:{self.dev_index}")
                     for _ in range(2)]
        self.copy_stream = torch.cuda.Stream(device=self.dev_index)
        self.copied = [torch.cuda.Event() for _ in range(2)]
        self.consumed = [torch.cuda.Event() for _ in range(2)]

    def __len__(self):
        return self.shape[0]

    def chunks(self):
        """Yield (r0, r1, device view) in order; copies run one chunk ahead on copy_stream."""
        N = self.shape[0]
        bounds = [(r0, min(N, r0 + self.chunk_rows)) for r0 in range(0, N, self.chunk_rows)]
        compute = torch.cuda.current_stream(self.dev_index)

        def issue(c):
            r0, r1 = bounds[c]
            b = c % 2
            with torch.cuda.stream(self.copy_stream):
                self.copy_stream.wait_event(self.consumed[b])
                self.bufs[b][: r1 - r0].copy_(self.X[r0:r1], non_blocking=True)
                self.copied[b].record(self.copy_stream)

        for b in range(2):  # both buffers start free
            self.consumed[b].record(compute)
        if bounds:
            issue(0)
        for c, (r0, r1) in enumerate(bounds):
            if c + 1 < len(bounds):
                issue(c + 1)
            b = c % 2
            compute.wait_event(self.copied[b])
            yield r0, r1, self.bufs[b][: r1 - r0]
            self.consumed[b].record(compute)
