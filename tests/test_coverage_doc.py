"""docs/COVERAGE.md must list every SURVEY.md §2.1 component and name only files that exist."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "cnmf_torch_amd")


def _read(rel):
    with open(os.path.join(ROOT, rel), encoding="utf-8") as f:
        return f.read()


def test_every_component_is_mapped():
    survey = _read("SURVEY.md")
    sec = survey.split("### 2.1", 1)[1].split("### 2.2", 1)[0]
    ids = set(re.findall(r"^\| (C\d+) \|", sec, re.M))
    assert len(ids) >= 40
    mapped = set(re.findall(r"^\| (C\d+) \|", _read("docs/COVERAGE.md"), re.M))
    assert ids <= mapped, sorted(ids - mapped)


def test_named_files_exist():
    doc = _read("docs/COVERAGE.md")
    missing = []
    for name in set(re.findall(r"`([\w/]+\.(?:py|hip|cpp|md))`", doc)):
        cands = [os.path.join(ROOT, name), os.path.join(PKG, name),
                 os.path.join(ROOT, "tests", name), os.path.join(ROOT, "csrc", "kernels", name),
                 os.path.join(ROOT, "csrc", "h5ad", name),
                 os.path.join(ROOT, "csrc", "io", name)]
        if not any(os.path.exists(c) for c in cands):
            missing.append(name)
    assert not missing, missing
