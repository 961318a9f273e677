"""Windowed and out-of-core sample sources for the gfx950 fit path.

The reference feeds windowed data through `util.WindowedDataset` (util.py:67-98): sample `idx`
is the window `X_untiled[idx + w0 : idx + w1]` with target `y[idx]`, for `idx` in
`usable_idx = arange(-w0, T - w1 + 1)`; its batch fits (standard_tensor_regression.py:478-620,
commented out) stack such windows into a dense (N, w1 - w0, ...) X.  Here the same samples
never get materialised:

* `windowed_view(X_untiled, y, win_range)` — every usable window, in `usable_idx` order, as one
  overlapping strided view (N, L, *F) with stride F along the sample axis.  X stays T x F in
  HBM; each kernel reads sample n at X + n*F (`tr_plan_set_x_stride`).
* `WindowedDataset` — the reference's `torch.utils.data.Dataset` (`usable_idx`, `ds[idx]`,
  `len(ds)` = series length, the `transform` / `target_transform` arguments) over that view.
* `make_WindowedDataloader` — the reference's random-minibatch loader over the usable windows
  (util.py:100-114), returning (dataloader, dataset, sampler) with `dataloader.sample_shape`.
* `HostStream` — an X kept in pinned host memory and streamed through two device buffers per
  iteration, for an X larger than the HBM one wants to spend.

The reference's general helpers (`set_device`, `squeeze_integers`) are not on the fit path and
are not provided.
"""
import numpy as np
import torch

__all__ = ["windowed_view", "WindowedDataset", "make_WindowedDataloader", "HostStream"]


def _usable_idx(T, win_range):
    w0, w1 = int(win_range[0]), int(win_range[1])
    return torch.arange(-w0, T - w1 + 1)


def windowed_view(X_untiled, y, win_range):
    """All usable windows of the series, as (Xw, yw): Xw[n] == X_untiled[n : n + L] is the window
    of idx = usable_idx[n] (idx + w0 == n), yw[n] == y[usable_idx[n]] (torch indexing, so a
    positive w0 wraps to the end of y exactly as the reference's `y_input[idx]` does).

    Xw is a zero-copy view of shape (T - L + 1, L, *F) and strides (F, F, *F-strides); only the
    N targets are gathered.  X_untiled is made contiguous first if it is not.
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
    y = torch.as_tensor(y)
    if y.shape[0] != T:  # checked on the host: an out-of-range gather would fault on the device
        raise ValueError(f"y must hold one target per series row: len(y) = {y.shape[0]}, series length {T}")
    feat = tuple(X_untiled.shape[1:])
    row = int(np.prod(feat)) if feat else 1
    Xw = X_untiled.as_strided((n, L) + feat, (row, row) + tuple(X_untiled.stride()[1:]))
    yw = y[_usable_idx(T, (w0, w1)).to(y.device)]
    return Xw, yw


class WindowedDataset(torch.utils.data.Dataset):
    """Indexable windows of an untiled series with the reference's sample numbering (util.py:67-98),
    a `torch.utils.data.Dataset` like the reference's.

    `ds[idx]` for idx in `ds.usable_idx` returns (window, target) as views into the strided
    `ds.windows` / gathered `ds.targets` (the tensors a fit takes directly).  `len(ds)` is the
    series length, as in the reference (util.py:78-79; `ds.n_windows` is the number of usable
    windows).  `transform` / `target_transform` are accepted and, as in the reference (which
    stores neither), not applied.  Deviation: an idx outside `usable_idx` raises IndexError, where
    the reference returns a truncated (or, for a negative start, wrapped) window.
    """

    def __init__(self, X_untiled, y_input, win_range, transform=None, target_transform=None):
        if len(X_untiled) != len(y_input):
            # (the reference's message: util.py:75-76)
            raise ValueError('RH: X and y must have same first dimension shape')
        self.X_untiled = X_untiled
        self.y_input = y_input
        self.win_range = (int(win_range[0]), int(win_range[1]))
        self.n_samples = int(len(y_input))
        self.windows, self.targets = windowed_view(X_untiled, y_input, self.win_range)
        self.usable_idx = _usable_idx(len(X_untiled), self.win_range)

    @property
    def n_windows(self):
        return int(self.windows.shape[0])

    def __len__(self):
        return self.n_samples

    def __getitem__(self, idx):
        n = int(idx) + self.win_range[0]
        if not 0 <= n < self.n_windows:
            raise IndexError(f"window index {int(idx)} is outside usable_idx "
                             f"[{int(self.usable_idx[0])}, {int(self.usable_idx[-1])}]")
        return self.windows[n], self.targets[n]


def make_WindowedDataloader(X, y, win_range=[-10, 10], batch_size=64, drop_last=True, **kwargs_dataloader):
    """The reference's minibatch loader over the usable windows (util.py:100-114): a
    `WindowedDataset`, a `SubsetRandomSampler` over its `usable_idx` and a `DataLoader` with the
    given batch size, `drop_last` and extra DataLoader arguments; `dataloader.sample_shape` =
    [batch_size] + one window's shape.  Returns (dataloader, dataset, sampler).  Each batch stacks
    its windows (the reference's host-side path); a fit over ALL windows takes
    `dataset.windows` / `dataset.targets` instead, which are never materialised."""
    dataset = WindowedDataset(X, y, win_range)
    sampler = torch.utils.data.SubsetRandomSampler(dataset.usable_idx, generator=None)
    dataloader = torch.utils.data.DataLoader(dataset, batch_size=batch_size, drop_last=drop_last, sampler=sampler,
                                             **kwargs_dataloader)
    dataloader.sample_shape = [dataloader.batch_size] + list(dataset[-win_range[0]][0].shape)
    return dataloader, dataset, sampler


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

    def range(self):
        """(max |x|, the smallest mean x^2 of a nonzero sample, min x) of the host X, computed once
        (the plan's X-form choice for its split kernels, Plan._x_form; the chunks are not measured
        one by one)."""
        if getattr(self, "_range", None) is None:
            a = self.X.reshape(self.shape[0], -1)
            if a.numel() == 0:
                self._range = (0.0, float("inf"), 0.0)
            else:
                mx = float("nan") if bool(torch.isnan(a).any()) else float(a.abs().max())
                ms = a.double().square().mean(dim=1)
                ms = ms[ms > 0]
                self._range = (mx, float(ms.min()) if ms.numel() else float("inf"), float(a.min()))
        return self._range

    @property
    def ndim(self):
        return len(self.shape)

    @property
    def dtype(self):
        return self.X.dtype

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

        # a buffer is free once the kernels of the last chunk that used it have run: the first
        # copies of an iteration wait only for those (an event never recorded is complete), so
        # they overlap the end of the previous iteration (its last chunks, reduction, Adam step)
        if bounds:
            issue(0)
        for c, (r0, r1) in enumerate(bounds):
            if c + 1 < len(bounds):
                issue(c + 1)
            b = c % 2
            compute.wait_event(self.copied[b])
            Xc = self.bufs[b][: r1 - r0]
            Xc._tr_stream = self  # (Plan._x_form takes the whole host X's range, not the chunk's)
            try:
                yield r0, r1, Xc
            finally:
                # also when the consumer raises or abandons the pass: the kernels it already
                # queued on this buffer must finish before a later pass copies into it
                self.consumed[b].record(compute)
