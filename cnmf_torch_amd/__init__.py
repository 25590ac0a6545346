"""cnmf_torch_amd -- MI355X-native consensus NMF (drop-in for aron0093/cNMF_torch).

Public API mirrors ``cnmf`` (src/cnmf/__init__.py:1-4 of the reference):
``cNMF``, ``Preprocess``, ``main``, ``save_df_to_npz``, ``load_df_from_npz``,
``__version__``.  The import of torch comes first so the HIP runtime is torch's.
"""
import torch  # noqa: F401  (load torch's HIP runtime before the native extension)

from .version import __version__
from .utils.io import load_df_from_npz, save_df_to_npz, save_df_to_text
from .api import cNMF
from .models.hvg import compute_tpm, get_highvar_genes, get_highvar_genes_sparse, get_mean_var
from .models.ols import efficient_ols_all_cols
from .models.refit import fit_H_online
from .models.nmf import run_nmf, run_nmf_batch
from .parallel.ledger import worker_filter
from .preprocess import Preprocess
from .cli import main

__all__ = ["cNMF", "Preprocess", "main", "save_df_to_npz", "load_df_from_npz", "save_df_to_text",
           "__version__", "compute_tpm", "get_highvar_genes", "get_highvar_genes_sparse",
           "get_mean_var", "efficient_ols_all_cols", "fit_H_online", "run_nmf", "run_nmf_batch",
           "worker_filter"]
