"""Repository hygiene (CPU): the reference-built checker libraries never travel to the GPU box.

oracle/_ref/ holds gcc builds of the reference's own C quantizers (oracle/Makefile `ref`), made
in the build container to generate and pin fixtures.  SURVEY.md (line 366, "What never leaves
this container") keeps reference sources, bytecode and .so files off the GPU box, so every path
under oracle/_ref must be excluded by a .gpurunignore pattern (tar --exclude semantics: a
pattern starting with ./ is anchored at the repository root, one without a slash matches a name
at any depth)."""
import fnmatch
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _patterns():
    with open(os.path.join(ROOT, ".gpurunignore")) as f:
        return [ln.strip() for ln in f if ln.strip() and not ln.startswith("#")]


def _excluded(rel, pats):
    parts = rel.split("/")
    for i in range(1, len(parts) + 1):
        prefix = "/".join(parts[:i])
        for p in pats:
            if p.startswith("./") and fnmatch.fnmatchcase(prefix, p[2:]):
                return True
            if "/" not in p and fnmatch.fnmatchcase(parts[i - 1], p):
                return True
            if not p.startswith("./") and "/" in p and fnmatch.fnmatchcase(prefix, p):
                return True
    return False


def test_reference_builds_are_gpurun_ignored():
    pats = _patterns()
    assert _excluded("oracle/_ref", pats), ".gpurunignore must exclude ./oracle/_ref"
    ref = os.path.join(ROOT, "oracle", "_ref")
    for d, _, files in os.walk(ref):
        for f in files:
            rel = os.path.relpath(os.path.join(d, f), ROOT)
            assert _excluded(rel, pats), f"{rel} would be pushed to the GPU box"


def test_product_libraries_are_not_gpurun_ignored():
    """The other way round: the built product and checker libraries the GPU tests load travel."""
    pats = _patterns()
    for rel in ("gguf-triton-kernel_amd/lib/libgguf_mmq.so", "gguf-triton-kernel_amd/lib/libgguf_quant.so",
                "oracle/liboracle.so", "tests/golden/golden_q8_0.npz"):
        assert not _excluded(rel, pats), rel
