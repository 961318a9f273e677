"""Known-answer tests (KATs) from the reference's own notebooks.

The reference ships no tests; its only executable evidence is two printed loss traces:
  KAT-1  demo_TensorRegression.ipynb (cells 5, 7, 8; printed trace at nb lines 217-219):
         CP_linear_regression, X (2000, 500, 500) fp64, rank 10, LBFGS (strong Wolfe), lambda 1e-5.
  KAT-2  demo_MultinomialTensorRegression.ipynb (cells 2, 4; printed trace at nb lines 152-187):
         CP_logistic_regression, 5 classes, rank 4, Adam lr 0.01 amsgrad, lambda 0.01, fp32 on CUDA.
The traces below are copied verbatim from the notebook outputs (data).  `kat_inputs` re-creates
the notebooks' synthetic inputs (seed 321; torch.rand + scipy savgol_filter) so they can be fed
to any implementation.  KAT-2 reproduces only if one extra multinomial make_BcpInit draw precedes
the model constructor (the notebook's execution count jumps 4 -> 6: an interrupted earlier run
of the cell consumed the RNG), and the notebook ran an older fit_Adam without class weights,
i.e. weights = ones(5).
"""
import numpy as np
import torch

KAT1_TRACE = np.array([560125.5196947237, 1699.8925874402807] + [0.041904340578888165] * 11)
KAT2_TRACE = np.array([
    1.8218674659729004, 1.7317867279052734, 1.6792151927947998, 1.6360952854156494, 1.6008062362670898,
    1.5716335773468018, 1.551900029182434, 1.534287691116333, 1.5129841566085815, 1.4906538724899292,
    1.4718546867370605, 1.4555275440216064, 1.4349761009216309, 1.4204165935516357, 1.4251134395599365,
    1.426369071006775, 1.4135684967041016, 1.3950250148773193, 1.3868310451507568, 1.3820008039474487,
    1.3758772611618042, 1.3679447174072266, 1.3580389022827148, 1.3488876819610596, 1.3384222984313965,
    1.325493574142456, 1.3122427463531494, 1.3004558086395264, 1.291756510734558, 1.284334659576416,
    1.2734110355377197, 1.264552354812622, 1.256840467453003, 1.2452030181884766, 1.2331522703170776,
    1.2235852479934692])


def _khatri_rao(mats):
    res = mats[0]
    for e in mats[1:]:
        res = torch.reshape(res[:, None, :] * e[None, :, :], (-1, res.shape[1]))
    return res


def _cp_to_tensor(w, F):
    return torch.reshape(torch.matmul(F[0] * w, _khatri_rao(F[1:]).T), [f.shape[0] for f in F])


def _underlying(n_samples=2000, n1=500, n2=500):
    import scipy.signal
    torch.manual_seed(321)
    np.random.seed(321)
    Xcp = [torch.rand(n_samples, 4) - 0.5,
           torch.vstack([torch.sin(torch.linspace(0, 140, n1)),
                         torch.cos(torch.linspace(2, 19, n1)),
                         torch.linspace(0, 1, n1),
                         torch.cos(torch.linspace(0, 17, n1)) > 0]).T,
           torch.tensor(scipy.signal.savgol_filter(np.random.rand(n2, 4), 15, 3, axis=0)) - 0.5]
    return Xcp


def kat_inputs(name):
    """(X, y) exactly as the notebook builds them (before the model constructor)."""
    w = torch.tensor(np.ones(4))
    if name == "kat1":
        Xcp = _underlying()
        Bcp = Xcp[1:]
        X_fake = _cp_to_tensor(w, Xcp)
        noisy = X_fake + torch.rand([2000, 500, 500]) / 100
        B = _cp_to_tensor(w, Bcp)
        y_hat = torch.reshape(torch.matmul(torch.reshape(noisy, (2000, -1)), torch.reshape(B, (-1, 1))), (2000,))
        del noisy
        X = X_fake - X_fake.mean(0)
        return X, y_hat
    if name == "kat2":
        Xcp = _underlying()
        Bcp = Xcp[1:] + [torch.rand(5, 4) - 0.5]
        X_fake = _cp_to_tensor(w, Xcp)
        B = _cp_to_tensor(w, Bcp)  # (500, 500, 5)
        Z = torch.reshape(torch.matmul(torch.reshape(X_fake, (2000, -1)), torch.reshape(B, (-1, 5))), (2000, 5))
        y = torch.argmax(torch.nn.functional.softmax(Z, dim=1), dim=1).numpy()
        X = X_fake.numpy()
        X = X - np.mean(X, axis=1)[:, None, :]
        return X, y
    raise ValueError(name)
