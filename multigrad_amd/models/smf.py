"""Stellar-mass-function example models (the reference's only workload), in PyTorch.

* :class:`MySMFModel` -- the test-suite model (reference
  ``tests/smf_example/smf_grad_descent.py:16-82``): params ``(log_shmrat, sigma_logsm)``,
  power-law halo masses, log-MSE loss against a target SMF.
* :class:`DocsSMFModel` -- the quick-start model (reference
  ``docs/source/notebooks/smf_gradient_descent.py:10-91``): params ``(log_f, log_sigma)``
  with ``sigma = 10**log_sigma`` and ``+1e-10`` inside the logs.

On a GPU the sumstats come from the fused HIP kernel (all bins in one pass over the
halos, ``csrc/smf.hip``); on CPU from the equivalent PyTorch expression.  Halos are
sharded across ranks with ``array_split`` exactly as in the reference, so the summed
sumstats are partition invariant.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import NamedTuple

import numpy as np
import torch

from ..ops.smf import PopulationShard, SmfBins, logmse_loss, smf_sumstats
from ..parallel.comm import get_world_comm
from .onepoint import OnePointModel

__all__ = ["ParamTuple", "load_halo_masses", "load_halo_masses_docs", "calc_smf_cdf",
           "calc_smf_bin", "MySMFModel", "DocsSMFModel", "TARGET_SUMSTATS", "make_test_data",
           "make_docs_data"]

# SMF at truth params=(-2.0, 0.2), 10_000 halos (reference tests/test_mpi.py:44-47)
TARGET_SUMSTATS = [
    2.30178721e-02, 1.69728529e-02, 1.16054425e-02, 7.10532581e-03,
    3.77187086e-03, 1.69136131e-03, 6.28149020e-04, 1.90466686e-04,
    4.66692982e-05, 9.17260695e-06]


class ParamTuple(NamedTuple):
    log_shmrat: float = -2.0
    sigma_logsm: float = 0.2


def _shard(arr: np.ndarray, comm) -> np.ndarray:
    comm = get_world_comm() if comm is None else comm
    return np.array_split(arr, comm.size)[comm.rank]


def load_halo_masses(num_halos=10_000, slope=-2, mmin=10.0 ** 10, qmax=0.95, comm=None):
    """Power-law halo masses (truncated so the SMF has a knee), this rank's shard."""
    q = np.linspace(0, qmax, num_halos, dtype=np.float32)
    mhalo = np.float32(mmin) * (1 - q) ** np.float32(1 / (slope + 1))
    return _shard(mhalo.astype(np.float32), comm)


def load_halo_masses_docs(num_halos=10_000, comm=None):
    """Halo masses between 1e10 and 1e11 (docs quick-start), this rank's shard."""
    quantile = np.linspace(0, 0.9, num_halos, dtype=np.float32)
    mhalo = np.float32(1e10) / (1 - quantile)
    return _shard(mhalo.astype(np.float32), comm)


def calc_smf_cdf(logsm, mean_logsm, sigma_logsm):
    return 0.5 * (1 + torch.special.erf((logsm - mean_logsm) / (np.sqrt(2) * sigma_logsm)))


def calc_smf_bin(params, logsm_low, logsm_high, volume, log_halo_masses):
    """One SMF bin (reference smf_grad_descent.py:38-48), PyTorch version."""
    params = ParamTuple(*params)
    mean_logsm = log_halo_masses + params.log_shmrat
    cdf_high = calc_smf_cdf(logsm_high, mean_logsm, params.sigma_logsm)
    cdf_low = calc_smf_cdf(logsm_low, mean_logsm, params.sigma_logsm)
    return torch.sum(cdf_high - cdf_low) / volume / (logsm_high - logsm_low)


def _device_default():
    # the fused HIP kernels are the default path whenever a GPU is present
    if torch.cuda.is_available():
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


class _SmfBase(OnePointModel):
    """Common plumbing: cached device shard + bins built from ``aux_data``."""

    _log_sigma = False
    _loss_eps = 0.0
    # the hooks ignore randkey (deterministic), so keyed runs may take the fused step
    engine_randkey_invariant = True

    def fused_step_engine(self, comm=None):
        """The cached fused GD / Adam / evaluation engine of this model on the GPU
        (:class:`multigrad_amd.engine.smf2.Smf2Engine`: one pass over the halos and one
        32-float exchange per step), or None (CPU, relative tails, > 16 bins)."""
        from ..engine.smf2 import Smf2Engine
        return Smf2Engine.for_model(self, comm)

    def _setup(self):
        dev = self.param_device()
        # rebuilt when the device or any aux_data entry is replaced (the cached fused step
        # engine follows the shard it was built on, engine/smf2.py)
        ad = self.aux_data or {}
        key = (str(dev), id(ad)) + tuple((k, id(ad[k])) for k in sorted(ad))
        if getattr(self, "_cache_key", None) != key:
            lhm = torch.as_tensor(np.asarray(self.aux_data["log_halo_masses"]), dtype=torch.float32)
            self._shard = PopulationShard(lhm, None, 1, device=dev)
            self._bins = SmfBins.make(np.asarray(self.aux_data["smf_bin_edges"], dtype=np.float64),
                                      float(self.aux_data["volume"]))
            self._target = torch.as_tensor(np.asarray(self.aux_data["target_sumstats"]),
                                           dtype=torch.float32, device=dev)
            self._cache_key = key
        return self._shard, self._bins

    def param_device(self) -> torch.device:
        if self.device is not None:
            return torch.device(self.device)
        return _device_default()

    def calc_partial_sumstats_from_params(self, params, randkey=None):
        shard, bins = self._setup()
        theta = torch.as_tensor(params).reshape(-1).to(shard.device)
        return smf_sumstats(theta, shard, bins, log_sigma=self._log_sigma)

    def calc_loss_from_sumstats(self, sumstats, sumstats_aux=None, randkey=None):
        self._setup()
        target = self._target.to(sumstats.device, sumstats.dtype)
        return logmse_loss(sumstats, target, self._loss_eps)


@dataclass(eq=False)
class MySMFModel(_SmfBase):
    """Test-suite SMF model: params ``(log_shmrat, sigma_logsm)`` (linear sigma)."""

    aux_data: dict = None
    loss_func_has_aux: bool = False

    _log_sigma = False
    _loss_eps = 0.0


@dataclass(eq=False)
class DocsSMFModel(_SmfBase):
    """Quick-start SMF model: params ``(log_f, log_sigma)``, ``sigma = 10**log_sigma``."""

    aux_data: dict = None

    _log_sigma = True
    _loss_eps = 1e-10


def make_test_data(num_halos=10_000, comm=None, device=None) -> dict:
    """aux_data of the reference test pipeline (tests/test_mpi.py:38-47)."""
    return dict(
        log_halo_masses=np.log10(load_halo_masses(num_halos, comm=comm)).astype(np.float32),
        smf_bin_edges=np.linspace(9, 10, 11),
        volume=10.0 * num_halos,
        target_sumstats=np.array(TARGET_SUMSTATS, dtype=np.float32),
    )


def make_docs_data(num_halos=10_000, true_params=(-2.0, -0.5), comm=None, device=None) -> dict:
    """aux_data of the docs quick-start (target = the SMF at the true parameters)."""
    lhm = np.log10(load_halo_masses_docs(num_halos, comm=comm)).astype(np.float32)
    data = dict(log_halo_masses=lhm, smf_bin_edges=np.linspace(9, 10, 11), volume=1.0,
                target_sumstats=np.ones(10, dtype=np.float32))
    model = DocsSMFModel(aux_data=data, comm=comm, device=device)
    data["target_sumstats"] = model.calc_sumstats_from_params(
        torch.tensor(true_params, dtype=torch.float32)).cpu().numpy()
    return data
