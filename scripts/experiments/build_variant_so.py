"""Build a variant of the kernels extension ``_C`` with extra compile flags on some sources, for
same-box A/Bs: the variant lands in ``tools_bin/variants/<name>/<_C .so name>`` (travels with the
gpurun snapshot; ``build/`` does not); ``scripts/so_ab.sh`` swaps it over the in-tree one between
runs.

    python scripts/experiments/build_variant_so.py depth3 kernels/attention.hip -DATTN_FP8_DEPTH3
    python scripts/experiments/build_variant_so.py ns1 norm.hip,rope_cache.hip,quant.hip -DPROBE_NS1

Reuses the in-tree build's objects for every other source (build it first: ``__graft_entry__``).
"""
import hashlib
import os
import shutil
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)

from distributed_llm_inference import _build as B  # noqa: E402


def main() -> None:
    name, flags = sys.argv[1], sys.argv[3:]
    src_rels = sys.argv[2].split(",")
    B.build_kernels()
    hipcc = shutil.which("hipcc") or os.path.join(B.ROCM, "bin", "hipcc")
    tcflags, ldflags = B._torch_flags()
    base = [hipcc, f"--offload-arch={B.ARCH}", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=fast",
            f"-I{B.CSRC}", "-Wno-unused-result", "-Wno-deprecated-declarations"]
    out_dir = os.path.join(REPO, "build", "variants", name)
    os.makedirs(out_dir, exist_ok=True)
    objs = []
    for s in B.KERNEL_SOURCES + B.TORCH_SOURCES:
        path = os.path.join(B.CSRC, s)
        if not os.path.exists(path):
            continue
        fl = base + (tcflags if s in B.TORCH_SOURCES else [])
        key = hashlib.sha1(" ".join(fl).encode()).hexdigest()[:8]
        obj = os.path.join(B.BUILD_DIR, s.replace("/", "_") + f".{key}.o")
        if any(s == r or s.endswith("/" + r) for r in src_rels):
            obj = os.path.join(out_dir, os.path.basename(s) + ".o")
            subprocess.run(fl + flags + ["-c", path, "-o", obj], check=True)
        objs.append(obj)
    so_dir = os.path.join(REPO, "tools_bin", "variants", name)
    os.makedirs(so_dir, exist_ok=True)
    so = os.path.join(so_dir, os.path.basename(B.kernels_so_path()))
    subprocess.run([hipcc, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", so] + objs + ldflags,
                   check=True)
    print(so)


if __name__ == "__main__":
    main()
