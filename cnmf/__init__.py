"""``import cnmf`` alias so code written against the reference package
(``from cnmf import cNMF, Preprocess``) runs unchanged on cnmf_torch_amd."""
from cnmf_torch_amd import *  # noqa: F401,F403
from cnmf_torch_amd import __version__, cNMF, Preprocess, main, load_df_from_npz, save_df_to_npz  # noqa: F401
