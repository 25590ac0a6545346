"""Replicate logs / manifest robustness."""
import json

import numpy as np
import pandas as pd
import pytest

from cnmf_torch_amd.utils.io import load_df_from_npz, save_arrays_npz_digest
from cnmf_torch_amd.utils.timing import append_jsonl_many, read_jsonl


def test_read_jsonl_skips_a_torn_tail(tmp_path):
    p = str(tmp_path / "log.jsonl")
    append_jsonl_many(p, [{"a": 1}, {"a": 2}])
    with open(p, "a") as fh:
        fh.write('{"a": 3, "b"')          # process killed mid-append
    with pytest.warns(UserWarning, match="undecodable"):
        recs = read_jsonl(p)
    assert recs == [{"a": 1}, {"a": 2}]


def test_npz_digest_matches_file_and_loads_as_dataframe(tmp_path):
    import hashlib

    p = str(tmp_path / "x.df.npz")
    data = np.arange(12, dtype=np.float32).reshape(3, 4)
    digest, size = save_arrays_npz_digest(p, {"data": data, "index": np.arange(1, 4),
                                              "columns": np.array(["g1", "g2", "g3", "g4"])})
    raw = open(p, "rb").read()
    assert hashlib.sha256(raw).hexdigest() == digest and len(raw) == size
    df = load_df_from_npz(p)
    assert list(df.columns) == ["g1", "g2", "g3", "g4"] and list(df.index) == [1, 2, 3]
    np.testing.assert_array_equal(df.values, data)


def test_verify_replicates_survives_torn_manifest(tmp_path):
    from cnmf_torch_amd import cNMF
    from cnmf_torch_amd.utils.synthetic import simulate_counts
    from cnmf_torch_amd.utils.io import save_df_to_npz

    X, cells, genes = simulate_counts(300, 400, 3, seed=0, sparse=False)
    counts = str(tmp_path / "counts.df.npz")
    save_df_to_npz(pd.DataFrame(X, index=cells, columns=genes), counts)
    obj = cNMF(output_dir=str(tmp_path), name="t")
    obj.prepare(counts, components=[3, 4], n_iter=2, seed=1, num_highvar_genes=200)
    obj.factorize(verbose=False)
    assert obj.verify_replicates() == []
    with open(obj.paths["replicate_manifest"], "a") as fh:
        fh.write('{"k": 3, "it')
    with pytest.warns(UserWarning):
        assert obj.verify_replicates() == []
    recs = read_jsonl(obj.paths["replicate_log"])
    assert sorted((r["k"], r["iter"]) for r in recs) == [(3, 0), (3, 1), (4, 0), (4, 1)]
    assert all(json.dumps(r) for r in recs)


def test_stored_zip_fast_path_is_a_standard_npz(tmp_path):
    import zipfile

    from cnmf_torch_amd.utils.io import npy_bytes, npz_bytes

    cols = np.array(["a", "bb", "ccc"])
    raw = npz_bytes({"data": np.ones((2, 3), np.float32), "index": np.arange(1, 3),
                     "columns": npy_bytes(cols)})
    p = tmp_path / "f.npz"
    p.write_bytes(raw)
    with zipfile.ZipFile(p) as zf:
        assert zf.testzip() is None
        assert sorted(zf.namelist()) == ["columns.npy", "data.npy", "index.npy"]
    with np.load(p, allow_pickle=False) as f:
        np.testing.assert_array_equal(f["columns"], cols)
        np.testing.assert_array_equal(f["data"], np.ones((2, 3), np.float32))


def test_npz_template_files_load_and_hash(tmp_path):
    import hashlib

    from cnmf_torch_amd.utils.io import NpzTemplate

    genes = np.array(["g%d" % i for i in range(50)])
    t = NpzTemplate({"columns": genes})
    for k in (3, 5):
        p = str(tmp_path / f"s{k}.df.npz")
        data = np.random.default_rng(k).random((k, 50)).astype(np.float32)
        digest, size = t.write(p, {"index": np.arange(1, k + 1), "data": data})
        raw = open(p, "rb").read()
        assert hashlib.sha256(raw).hexdigest() == digest and len(raw) == size
        df = load_df_from_npz(p)
        np.testing.assert_array_equal(df.values, data)
        assert list(df.index) == list(range(1, k + 1)) and list(df.columns) == list(genes)


def test_native_spectra_batch_reader(tmp_path):
    """The native reader (csrc/io/npzio.cpp) returns exactly what the native writer wrote,
    and declines (None -> numpy path) files it does not handle: deflated members,
    gene-name bytes that differ from the first file's."""
    import numpy as np
    import pandas as pd

    from cnmf_torch_amd.utils import io as cio

    if cio._npzio is None:
        pytest.skip("native npz extension not built")
    G = 300
    cols = np.array([f"g{i}" for i in range(G)])
    ks = [5, 7, 5]
    offs = [0, 5, 12]
    data = np.random.default_rng(0).random((17, G)).astype(np.float32)
    paths = [str(tmp_path / f"r{i}.df.npz") for i in range(3)]
    cio.write_spectra_batch(paths, data, offs, ks, cols)
    got = cio.read_spectra_batch(paths)
    assert got is not None
    np.testing.assert_array_equal(got[0], data)
    assert got[1] == ks and list(got[2]) == list(cols)
    # numpy reads the same files to the same arrays
    with np.load(paths[1]) as f:
        np.testing.assert_array_equal(f["data"], data[5:12])
    # other gene-name bytes -> declined
    other = [str(tmp_path / "o.df.npz")]
    cio.write_spectra_batch(other, data[:5], [0], [5], np.array([f"x{i}" for i in range(G)]))
    assert cio.read_spectra_batch(paths + other) is None
    # a deflated file (e.g. written by the original cnmf) -> declined
    cio.save_df_to_npz(pd.DataFrame(data[:5], columns=cols), paths[0], level=6)
    assert cio.read_spectra_batch(paths) is None


def test_native_tsv_writer_is_byte_identical_to_pandas(tmp_path):
    """save_df_to_text's native writer (npzio.cpp write_tsv) produces the same bytes as
    DataFrame.to_csv(sep='\\t') -- float64 repr / float32 str rules, NaN as '', inf,
    -0.0, integral values, every decade -- and leaves other frames to pandas."""
    import numpy as np
    import pandas as pd

    from cnmf_torch_amd.utils import io as cio

    rng = np.random.default_rng(1)
    with np.errstate(over="ignore"):
        mags = 10.0 ** rng.uniform(-320, 320, 7000)
    vals = np.concatenate([mags * rng.choice([-1, 1], mags.size),
                           rng.random(7000) * 10.0 ** rng.integers(-7, 18, 7000),
                           [0.0, -0.0, np.nan, np.inf, -np.inf, 1e-4, 1e16, 1e-5, 3.0,
                            0.0001, 12345678901234567.0, 5e-324, 123456789.125]])
    vals = vals[: (vals.size // 8) * 8].reshape(-1, 8)
    for dt in (np.float64, np.float32):
        with np.errstate(over="ignore"):
            df = pd.DataFrame(vals.astype(dt), index=[f"cell{i}" for i in range(len(vals))],
                              columns=[f"g{j}" for j in range(8)])
        for name in (None, "idx"):
            df.index.name = name
            assert cio._tsv_native_args(df) is not None
            a, b = tmp_path / "a.txt", tmp_path / "b.txt"
            cio.save_df_to_text(df, a)
            df.to_csv(b, sep="\t")
            assert a.read_bytes() == b.read_bytes()
    mixed = pd.DataFrame({"a": [1, 2], "b": [0.5, 1.5]})
    assert cio._tsv_native_args(mixed) is None
    quoted = pd.DataFrame([[1.0]], index=['x"y'], columns=["c"])
    assert cio._tsv_native_args(quoted) is None
    cio.save_df_to_text(quoted, tmp_path / "q.txt")
    assert (tmp_path / "q.txt").read_text() == quoted.to_csv(sep="\t")


def test_row_block_h5ad_writer_holds_one_block_at_a_time(tmp_path):
    """write_h5ad_row_blocks (the sharded prepare's rank-0 writer) writes the same h5ad as
    write_h5ad of the stacked matrix, CSR and dense, and releases every row block before
    it asks for the next one -- so rank 0 never holds more than one peer block."""
    import gc
    import weakref

    import numpy as np
    import pandas as pd
    import scipy.sparse as sp

    from cnmf_torch_amd.utils.h5ad import read_h5ad, write_h5ad_row_blocks

    rng = np.random.default_rng(0)
    X = sp.random(70, 12, density=0.3, random_state=1, format="csr", dtype=np.float64)
    obs = pd.DataFrame(index=[f"c{i}" for i in range(70)])
    var = pd.DataFrame(index=[f"g{j}" for j in range(12)])
    cuts = [0, 20, 21, 55, 70]
    for sparse in (True, False):
        live = []

        def blocks():
            for a, b in zip(cuts[:-1], cuts[1:]):
                gc.collect()
                assert all(r() is None for r in live), "a previous block is still held"
                blk = X[a:b] if sparse else X[a:b].toarray()
                arr = blk.data if sparse else blk
                live.append(weakref.ref(arr))
                yield obs.iloc[a:b], blk
                del blk, arr       # (this generator's own references)
        path = str(tmp_path / f"x{int(sparse)}.h5ad")
        write_h5ad_row_blocks(path, 70, var, blocks(), sparse, np.float64, X.nnz)
        got = read_h5ad(path)
        gx = got.X.toarray() if sp.issparse(got.X) else got.X
        np.testing.assert_array_equal(gx, X.toarray())
        assert sp.issparse(got.X) == sparse
        assert list(got.obs.index) == list(obs.index) and list(got.var.index) == list(var.index)


def test_parallel_deflate_npz_is_a_standard_npz(tmp_path, monkeypatch):
    """Members >= the parallel threshold are deflated in independent full-flushed chunks
    on threads: the archive is a standard ZIP_DEFLATED npz (zipfile's CRC check, np.load,
    load_df_from_npz) with the same contents as the one-thread writer."""
    import zipfile

    import numpy as np
    import pandas as pd

    from cnmf_torch_amd.utils import io as cio

    monkeypatch.setattr(cio, "_PAR_DEFLATE_MIN", 1 << 16)
    monkeypatch.setattr(cio, "_PAR_DEFLATE_CHUNK", 1 << 14)
    rng = np.random.default_rng(3)
    df = pd.DataFrame(np.round(rng.random((3000, 7)), 3), index=[f"c{i}" for i in range(3000)],
                      columns=[f"g{j}" for j in range(7)])
    fn = str(tmp_path / "p.npz")
    cio.save_df_to_npz(df, fn)
    with zipfile.ZipFile(fn) as z:
        assert z.testzip() is None
        assert all(i.compress_type == zipfile.ZIP_DEFLATED for i in z.infolist())
    pd.testing.assert_frame_equal(cio.load_df_from_npz(fn, allow_pickle_fallback=False), df)
    with np.load(fn, allow_pickle=False) as f:
        np.testing.assert_array_equal(f["data"], df.values)
