"""fp64 torch reference backend for the GLM aggregation kernels (K1-K5 of SURVEY.md §2.8).

This is the numerical spec every HIP kernel is tested against, and the CPU execution path (the analogue of
Spark ``local[*]``). It mirrors the per-row aggregator semantics of
``photon-lib/.../function/glm/ValueAndGradientAggregator.scala:132-153`` (value/grad),
``HessianVectorAggregator.scala:96-121`` (Hv) and ``HessianDiagonalAggregator.scala:51-61`` (Hdiag), but as
whole-shard sparse matrix products instead of a per-record fold.
"""
from __future__ import annotations

from typing import Optional

import warnings

import numpy as np
import scipy.sparse as sp
import torch

warnings.filterwarnings("ignore", message="Sparse CSR tensor support is in beta state")

from ..data.matrix import LabeledData


def _to_torch_csr(m: sp.csr_matrix, device, dtype=torch.float64) -> torch.Tensor:
    m = m.tocsr()
    return torch.sparse_csr_tensor(
        torch.from_numpy(m.indptr.astype(np.int64)),
        torch.from_numpy(m.indices.astype(np.int64)),
        torch.from_numpy(m.data.astype(np.float64)),
        size=m.shape,
        dtype=dtype,
    ).to(device)


class GLMComputable:
    """Interface of a row shard that can evaluate GLM aggregates.

    All vectors are fp64 torch tensors on ``self.device``; scalars are python floats.
    """

    n_rows: int
    dim: int
    device: torch.device

    def value_grad_sums(self, loss, w_eff, margin_shift: float):
        """Return ``(F, S, G)``: F = sum w_i l(z_i), S = sum w_i l'(z_i), G = sum w_i l'(z_i) x_i."""
        raise NotImplementedError

    def hv_sums(self, loss, w_eff, margin_shift: float, v_eff, v_shift: float):
        """Return ``(H, P)``: e_i = w_i l''(z_i) (x_i.v_eff - v_shift); H = sum e_i x_i, P = sum e_i."""
        raise NotImplementedError

    def hdiag_sums(self, loss, w):
        """Return sum_i w_i l''(x_i.w + o_i) x_i^2 (raw coefficients, no normalisation)."""
        raise NotImplementedError

    def margins(self, w, margin_shift: float = 0.0, with_offsets: bool = False):
        """x_i . w (+ shift) (+ o_i)."""
        raise NotImplementedError

    def matvec(self, w):
        """X w."""
        raise NotImplementedError

    def rmatvec(self, r, square: bool = False, build_multi: bool = True):
        """X^T r (``square``: (X.X)^T r)."""
        raise NotImplementedError

    def count(self) -> int:
        return self.n_rows


class TorchGLMData(GLMComputable):
    """Reference backend: torch sparse CSR (X and X^T) in fp64 on any device."""

    def __init__(self, data: LabeledData, device="cpu"):
        self.device = torch.device(device)
        self.n_rows, self.dim = data.x.shape
        self.x = _to_torch_csr(data.x, self.device)
        self.xt = _to_torch_csr(data.x.T.tocsr(), self.device)
        self.x2t = _to_torch_csr(data.x.multiply(data.x).T.tocsr(), self.device)
        self.y = torch.from_numpy(data.y).to(self.device)
        self.o = torch.from_numpy(data.offsets).to(self.device)
        self.wt = torch.from_numpy(data.weights).to(self.device)

    def _xv(self, w):
        if self.n_rows == 0:
            return torch.zeros(0, dtype=torch.float64, device=self.device)
        return torch.mv(self.x, w.to(self.device, torch.float64))

    def _xtv(self, r):
        if self.n_rows == 0:
            return torch.zeros(self.dim, dtype=torch.float64, device=self.device)
        return torch.mv(self.xt, r)

    def margins(self, w, margin_shift: float = 0.0, with_offsets: bool = False):
        z = self._xv(w) + margin_shift
        return z + self.o if with_offsets else z

    def matvec(self, w):
        return self._xv(w)

    def rmatvec(self, r, square: bool = False, build_multi: bool = True):
        r = torch.as_tensor(r, dtype=torch.float64, device=self.device)
        if self.n_rows == 0:
            return torch.zeros(self.dim, dtype=torch.float64, device=self.device)
        m = self.x2t if square else self.xt
        return (m @ r.unsqueeze(1)).squeeze(1)

    def value_grad_sums(self, loss, w_eff, margin_shift):
        z = self._xv(w_eff) + margin_shift + self.o
        l, dl = loss.loss_and_dz(z, self.y)
        r = self.wt * dl
        return float(torch.sum(self.wt * l)), float(torch.sum(r)), self._xtv(r)

    def zero_point_sums(self, loss, margin_shift):
        """[F, S, ||c||^2, ||X||_F^2] at w = 0 (see DeviceGLMData.zero_point_sums)."""
        l, dl = loss.loss_and_dz(self.o + margin_shift, self.y)
        c = self.wt * dl
        xsq = float(torch.sum(self.x.values() ** 2)) if self.n_rows else 0.0
        return [float(torch.sum(self.wt * l)), float(torch.sum(c)), float(torch.dot(c, c)), xsq]

    def hv_sums(self, loss, w_eff, margin_shift, v_eff, v_shift):
        z = self._xv(w_eff) + margin_shift + self.o
        u = self._xv(v_eff) - v_shift
        if getattr(self, "_track_u", False):
            self._u = u
        e = self.wt * loss.dzz(z, self.y) * u
        return self._xtv(e), float(torch.sum(e))

    def hdiag_sums(self, loss, w):
        z = self._xv(w) + self.o
        d = self.wt * loss.dzz(z, self.y)
        if self.n_rows == 0:
            return torch.zeros(self.dim, dtype=torch.float64, device=self.device)
        return torch.mv(self.x2t, d)

    def row_losses(self, loss, w_eff, margin_shift=0.0):
        z = self._xv(w_eff) + margin_shift + self.o
        l, _ = loss.loss_and_dz(z, self.y)
        return l

    # margin-space line search (see GLMObjective.margin_line_search); fp64 reference of ls_eval_kernel
    def ls_begin(self, w0_eff, shift0, d_eff, d_shift, t0: float = 1.0, loss=None) -> bool:
        self._z0 = self.margins(w0_eff, shift0, True)
        self._zd = self.margins(d_eff, d_shift, False)
        return True

    def ls_eval(self, loss, t: float):
        l, dl = loss.loss_and_dz(self._z0 + t * self._zd, self.y)
        return float(torch.sum(self.wt * l)), float(torch.sum(self.wt * dl * self._zd))

    def ls_finish_sums(self, loss, t: float, w_eff, shift, need_s: bool = True):
        self._track_u = False
        z = self._z0 + t * self._zd
        l, dl = loss.loss_and_dz(z, self.y)
        r = self.wt * dl
        return float(torch.sum(self.wt * l)), float(torch.sum(r)), self._xtv(r)

    # TRON trial in margin space (see DeviceGLMData.step_begin): fp64 reference
    def step_begin(self, w_eff, shift) -> bool:
        self._z0 = self.margins(w_eff, shift, True)
        self._zd = torch.zeros_like(self._z0)
        self._track_u = True
        return True

    def step_add(self, alpha: float):
        self._zd = self._zd + float(alpha) * self._u

    def set_offsets(self, offsets):
        self.o = torch.as_tensor(offsets, dtype=torch.float64).to(self.device)

    def set_weights(self, weights):
        self.wt = torch.as_tensor(weights, dtype=torch.float64).to(self.device)
