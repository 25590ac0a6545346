"""Generate the regression fixtures used by tests/test_reproducibility.py (C41).

The reference downloads two golden tarballs (download_pytest_data.py:35-69): a simulated
counts table and a PBMC h5ad, each with the outputs of a reference run.  This machine
has no network and the golden outputs of *this* framework are what a regression test
must pin, so the inputs are simulated deterministically (utils/synthetic.py) and the
golden outputs come from a CPU float64-oracle run of our own pipeline:

    python tools/make_test_data.py            # writes tests/data/golden/<dataset>/...

Only the files the test compares are kept (merged spectra are the consensus input, as
in the reference test, plus the consensus / prepare outputs).
"""
import argparse
import os
import shutil
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import pandas as pd  # noqa: E402

from cnmf_torch_amd import cNMF, save_df_to_npz  # noqa: E402
from cnmf_torch_amd.utils.anndata_lite import AnnData  # noqa: E402
from cnmf_torch_amd.utils.h5ad import write_h5ad  # noqa: E402
from cnmf_torch_amd.utils.synthetic import simulate_counts  # noqa: E402

DATASETS = {
    # mirrors tests/test_reproducibility.py of the reference: text counts, K 5..7, 15 iter
    "simulated_example_data": dict(kind="txt", cells=600, genes=400, programs=6, seed=11,
                                   k_values=[5, 6, 7], n_iter=15, nhvg=300,
                                   consensus=[(6, 0.1)]),
    # sparse h5ad input, two consensus runs
    "example_sparse_h5ad": dict(kind="h5ad", cells=700, genes=500, programs=7, seed=12,
                                k_values=[6, 7, 8], n_iter=15, nhvg=300,
                                consensus=[(7, 0.1), (8, 0.1)]),
}
SEED = 14
GOLDEN_KEYS = ["consensus_spectra", "consensus_usages", "gene_spectra_score",
               "gene_spectra_tpm", "starcat_spectra"]
PREPARE_KEYS = ["normalized_counts", "nmf_replicate_parameters", "nmf_run_parameters",
                "nmf_genes_list", "tpm", "tpm_stats"]


def write_counts(cfg: dict, out_dir: str) -> str:
    X, cells, genes = simulate_counts(cfg["cells"], cfg["genes"], cfg["programs"],
                                      seed=cfg["seed"], sparse=cfg["kind"] == "h5ad")
    os.makedirs(out_dir, exist_ok=True)
    if cfg["kind"] == "txt":
        fn = os.path.join(out_dir, "filtered_counts.txt")
        pd.DataFrame(X, index=cells, columns=genes).to_csv(fn, sep="\t")
    else:
        fn = os.path.join(out_dir, "counts.h5ad")
        write_h5ad(fn, AnnData(X=X, obs=pd.DataFrame(index=cells), var=pd.DataFrame(index=genes)))
    return fn


def run(cfg: dict, name: str, out_dir: str, counts_fn: str) -> cNMF:
    obj = cNMF(output_dir=out_dir, name=name)
    obj.prepare(counts_fn, components=cfg["k_values"], n_iter=cfg["n_iter"],
                num_highvar_genes=cfg["nhvg"], seed=SEED)
    obj.factorize(device="cpu")
    obj.combine()
    for k, thr in cfg["consensus"]:
        obj.consensus(k, density_threshold=thr, show_clustering=False)
    return obj


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "tests", "data", "golden"))
    a = ap.parse_args()
    for ds, cfg in DATASETS.items():
        with tempfile.TemporaryDirectory() as tmp:
            counts = write_counts(cfg, tmp)
            obj = run(cfg, ds, tmp, counts)
            dst = os.path.join(a.out, ds)
            if os.path.isdir(dst):
                shutil.rmtree(dst)
            os.makedirs(os.path.join(dst, "cnmf_tmp"))

            def keep(path):
                rel = os.path.relpath(path, os.path.join(tmp, ds))
                shutil.copy(path, os.path.join(dst, rel))

            for k in cfg["k_values"]:
                keep(obj.paths["merged_spectra"] % k)
            for key in GOLDEN_KEYS:
                for k, thr in cfg["consensus"]:
                    keep(obj.paths[key] % (k, str(thr).replace(".", "_")))
            for key in PREPARE_KEYS:
                if key not in ("normalized_counts", "tpm"):
                    keep(obj.paths[key])
            print(f"wrote {dst}")


if __name__ == "__main__":
    main()
