"""Print each kernel's instruction stream in device assembly, compressed to the instructions that
shape a ping-pong GEMM main loop (MFMA, s_barrier, ds_read, LDS-DMA, s_waitcnt, s_setprio, loop
labels), runs collapsed to `name xN`.  Used to check that the compiler kept every quadrant's MFMAs
between their barriers (it sank all of them to the loop's end in the fp8 kernel once).

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=fast -Idistributed_llm_inference/csrc \
          --cuda-device-only -S distributed_llm_inference/csrc/kernels/gemm_tile.hip -o /tmp/gt.s
    python scripts/isa_phase_summary.py /tmp/gt.s [kernel-substring]
"""
import re
import sys

KEEP = ("v_mfma", "s_barrier", "ds_read", "global_load", "buffer_load", "v_cvt_scalef32_pk_bf16_fp8", "v_cvt_pk_bf16", "s_waitcnt", "s_setprio",
        "s_cbranch")


def main(path, want=""):
    kern, seq = None, []

    def flush():
        if kern and want in kern and any(s == "MFMA" for s, _ in seq):
            print(f"== {kern}")
            print(" ".join(f"{s}x{n}" if n > 1 else s for s, n in seq))
            print()

    for line in open(path):
        m = re.match(r"^(_Z\w+):(\s|$)", line)
        if m:
            flush()
            kern, seq = m.group(1), []
            continue
        if re.match(r"^\.LBB\d+_\d+:.*Loop Header", line):
            seq.append(("[LOOP]", 1))
            continue
        tok = line.split()
        if not tok or tok[0].startswith((";", ".")):
            continue
        op = tok[0]
        if not op.startswith(KEEP):
            continue
        if op == "s_waitcnt":
            op = "wait(" + " ".join(tok[1:]) + ")"
        elif op.startswith("v_mfma"):
            op = "MFMA"
        if seq and seq[-1][0] == op:
            seq[-1] = (op, seq[-1][1] + 1)
        else:
            seq.append((op, 1))
    flush()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
