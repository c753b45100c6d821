"""The package's environment surface stays small and documented: every
``DLI_*`` name in the package sources, bench.py, distribute and __graft_entry__.py is listed in
docs/env.md, and there are at most 20 of them.  Kernel choices are KernelPolicy fields."""
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PAT = re.compile(r"\bDLI_[A-Z0-9_]+\b")


def _package_names():
    names = {}
    roots = [os.path.join(REPO, "distributed_llm_inference")]
    files = [os.path.join(REPO, f) for f in ("bench.py", "distribute", "__graft_entry__.py")]
    for root in roots:
        for d, _, fs in os.walk(root):
            if "__pycache__" in d:
                continue
            files += [os.path.join(d, f) for f in fs
                      if f.endswith((".py", ".hip", ".h", ".cpp", ".csv"))]
    for f in files:
        with open(f, errors="replace") as fh:
            for n in PAT.findall(fh.read()):
                names.setdefault(n, set()).add(os.path.relpath(f, REPO))
    return names


def _documented():
    with open(os.path.join(REPO, "docs", "env.md")) as fh:
        text = fh.read()
    table = text.split("## Environment variables", 1)[1].split("Retired in round 5", 1)[0]
    return set(re.findall(r"`(DLI_[A-Z0-9_]+)`", table))


def test_every_env_name_is_documented():
    names, doc = _package_names(), _documented()
    missing = {n: sorted(fs) for n, fs in names.items() if n not in doc}
    assert not missing, f"DLI_* names used but not listed in docs/env.md: {missing}"


def test_env_surface_is_small_and_has_no_stale_docs():
    names, doc = _package_names(), _documented()
    assert len(names) <= 20, sorted(names)
    stale = doc - set(names)
    assert not stale, f"docs/env.md lists names the package no longer reads: {sorted(stale)}"


def test_kernel_policy_overrides_parse_and_reject_unknown_fields():
    from distributed_llm_inference.config import KernelPolicy
    p = KernelPolicy().with_overrides("gemm4=1, library_gemms=auto ,fp8_gemm4=gate_up+down")
    assert p.gemm4 and p.library_gemms is None
    assert p.fp8_on_gemm4("down") and not p.fp8_on_gemm4("qkv")
    assert not p.with_overrides("gemm4=0").fp8_on_gemm4("down")   # gemm4 off: nothing on it
    assert KernelPolicy(fp8_gemm4="all").fp8_on_gemm4("o")
    with pytest.raises(ValueError, match="unknown kernel policy field"):
        KernelPolicy().with_overrides("gemm5=1")
    with pytest.raises(ValueError):
        KernelPolicy(fp8_gemm4="lm_head")


def test_kernel_policy_env_and_context(monkeypatch):
    from distributed_llm_inference import ops
    from distributed_llm_inference.config import KernelPolicy
    monkeypatch.setenv("DLI_KERNELS", "bf16_partials=0")
    ops._POLICY = None
    assert not ops.policy().bf16_partials and ops.policy().gemm4
    # an installed policy keeps the env override on top
    ops.set_policy(KernelPolicy(gemm4=False))
    assert not ops.policy().gemm4 and not ops.policy().bf16_partials
    with ops.kernel_policy(gemv=False):
        assert not ops.policy().gemv
    assert ops.policy().gemv
