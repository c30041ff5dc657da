"""Check a kernel's ISA for asm LDS reads whose destination registers are read or written before
an lgkmcnt wait covers them (csrc/noise_mlp.hip solo::, the RULE at lds_f4).  The compiler treats an
inline-asm ds_read's output as available at once; only a tied s_waitcnt keeps the registers from
being reused while the data is in flight.

    python tools/asm_hazard.py [kernel-symbol-substring]   (builds noise_mlp.hip's ISA with hipcc)

Exit status 1 when a hazard is found."""
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def regs(tok):
    """VGPRs and AGPRs named in an operand string, as ('v'|'a', index)"""
    out = set()
    for m in re.finditer(r"\b([va])\[(\d+):(\d+)\]", tok):
        out |= {(m.group(1), i) for i in range(int(m.group(2)), int(m.group(3)) + 1)}
    for m in re.finditer(r"\b([va])(\d+)\b", tok):
        out.add((m.group(1), int(m.group(2))))
    return out


def scan(lines):
    pending = {}  # register -> index of the ds_read that targets it
    issues = []
    for n, l in enumerate(lines):
        if l.startswith("ds_read"):
            for r in regs(l.split(None, 1)[1].split(",")[0]):
                pending[r] = n
            continue
        if l.startswith("s_waitcnt") and "lgkmcnt" in l:
            k = int(re.search(r"lgkmcnt\((\d+)\)", l).group(1))
            order = sorted(set(pending.values()))
            keep = set(order[-k:]) if k > 0 else set()   # LDS operations complete in order
            pending = {r: i for r, i in pending.items() if i in keep}
            continue
        if not l or l[0] in ";.":
            continue
        if l.startswith("s_"):   # scalar instructions and branches name no VGPR we track
            if l.startswith(("s_cbranch", "s_branch", "s_endpgm")):
                pending.clear()  # block boundary: stay local (the kernel's reads do not cross one)
            continue
        parts = l.split(None, 1)
        if len(parts) < 2:
            continue
        ops = parts[1].split(",")
        used = set()
        for o in ops:
            used |= regs(o)
        hit = used & set(pending)
        if hit:
            r = min(hit)
            issues.append((n, l, lines[pending[r]]))
    return issues


def main():
    want = sys.argv[1] if len(sys.argv) > 1 else "noise_mlp_solo_kernel"
    csrc = os.path.join(REPO, "pointcloud_style_transfer_amd", "csrc")
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "k.s")
        cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-I", os.path.join(REPO, "include"),
               "-I", csrc, "-mno-amdgpu-ieee", "-fno-honor-nans", "--cuda-device-only", "-S", "-o", out,
               os.path.join(csrc, "noise_mlp.hip")] + sys.argv[2:]
        subprocess.run(cmd, check=True, capture_output=True)
        text = open(out).read()
    bad = 0
    for m in re.finditer(r"^(_Z\S*%s\S*):" % re.escape(want), text, re.M):
        body = text[m.start():text.find(".Lfunc_end", m.start())]
        lines = [x.strip() for x in body.split("\n")]
        issues = scan(lines)
        print(f"{m.group(1)[:60]}: {len(issues)} hazard(s)")
        for n, l, src in issues[:10]:
            print(f"  line {n}: {l}   <- in flight from: {src}")
        bad += len(issues)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
