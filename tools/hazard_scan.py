"""Scan gfx950 device assembly for the wide-store data hazard.

A VMEM store of more than 64 bits reads its data VGPRs after it issues; on gfx940/950 a VALU
write of those VGPRs needs 2 wait states behind the store.  LLVM's hazard recognizer
(GCNHazardRecognizer::createsVALUHazard) inserts them for FLAT / GLOBAL stores and for MUBUF
stores whose soffset is a constant, but EXEMPTS a MUBUF store with a register soffset: it then
schedules VALU writes of the data VGPRs straight behind the store (checked with a test kernel:
soffset 0 -> `s_nop 1`, soffset s0 -> nothing).  Both r03 wrong-result events had exactly that
code: the bf16 study variant of k_col2<32> (non-deterministic, `buffer_store_dwordx4 v[0:3], ...,
s1 offen nt` -> `v_bfe_u32 v0, ...`; profiles/archive/r03/bf16_determinism_r03f.txt) and the ITER = 1
k_col2<16> build (wrong B rows, `buffer_store_dwordx4 v[32:35], ..., s11 offen nt` ->
`v_add_f32_e32 v32, ...`; profiles/archive/r03/kcol2_iter1_anomaly.txt), and neither hazard shows in
the builds that were exact.

Two rules, both must hold in every product kernel:
  * structural: no MUBUF store wider than 64 bits with a register soffset (the product passes
    soffset 0 and folds the offset into voffset, so LLVM's recognizer covers every such store);
  * window: no instruction that writes a VGPR overlapping a >64-bit store's data within the
    next 2 wait states (an instruction is 1, `s_nop N` is N + 1).

    python tools/hazard_scan.py            # compiles csrc/*.hip to assembly (-S), scans, exit 1 on any
    python tools/hazard_scan.py FILE.s ... # scan given assembly files
"""
import glob
import os
import re
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "binary-hologram-reinforcement-learning_amd", "csrc")
STORE = re.compile(r"^(buffer|global|flat|scratch)_store_(dwordx3|dwordx4|b96|b128)\s+(.*)$")
# first operand of an instruction when it is a VGPR (v7 / v[4:7]): the destination of VALU ops
VDST = re.compile(r"^(v_\w+)\s+(?:v(\d+)\b|v\[(\d+):(\d+)\])")
FUNC = re.compile(r"^(_Z\w+):")
WAIT_STATES = 2          # gfx940+ (LLVM: VALUWaitStates = hasGFX940Insts() ? 2 : 1)


def _instrs(path):
    """(line number, text, function) of every instruction, labels / directives / comments dropped."""
    func = None
    for k, raw in enumerate(open(path)):
        l = raw.split(";")[0].strip()
        if not l:
            continue
        m = FUNC.match(l)
        if m:
            func = m.group(1)
            continue
        if l[0] == "." or l.endswith(":"):
            continue
        yield k + 1, l, func


def scan(path, window=WAIT_STATES):
    """[(function, line, store, offender, rule)] for every violation in an assembly file."""
    hits = []
    ins = list(_instrs(path))
    for n, (line, l, func) in enumerate(ins):
        m = STORE.match(l)
        if not m:
            continue
        ops = [o.strip() for o in m.group(3).split(",")]
        regs = re.findall(r"v\[(\d+):(\d+)\]", m.group(3))
        if not regs:
            continue
        if m.group(1) == "buffer":
            lo, hi = map(int, regs[0])                       # buffer_store vdata, vaddr, srsrc, soffset
            soff = ops[3].split()[0] if len(ops) >= 4 and ops[3] else ""
            if re.fullmatch(r"s\d+", soff):
                hits.append((func, line, l, soff, "register-soffset"))
        else:
            lo, hi = map(int, regs[-1] if m.group(1) in ("global", "flat") else regs[0])
        budget = window
        for line2, l2, _ in ins[n + 1:]:
            if budget <= 0 or l2.startswith("s_endpgm") or l2.startswith("s_branch") \
                    or l2.startswith("s_cbranch") or l2.startswith("s_setpc"):
                break
            nop = re.match(r"^s_nop\s+(\d+)", l2)
            if nop:
                budget -= int(nop.group(1)) + 1
                continue
            d = VDST.match(l2)
            if d:
                dlo = int(d.group(2) or d.group(3))
                dhi = int(d.group(4)) if d.group(4) else dlo
                if "_b64" in d.group(1) or "_f64" in d.group(1) or "_u64" in d.group(1) \
                        or "_i64" in d.group(1):
                    dhi = max(dhi, dlo + 1)
                if not (dhi < lo or dlo > hi):
                    hits.append((func, line, l, l2, "data-overwrite"))
                    break
            budget -= 1
    return hits


def compile_all(outdir, srcs=None, defines=()):
    srcs = srcs or sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

    def one(src):
        out = os.path.join(outdir, os.path.basename(src) + ".s")
        subprocess.run([hipcc, "-O3", "-std=c++17", "-fno-slp-vectorize", "--offload-arch=gfx950",
                        "-I" + os.path.join(ROOT, "include"), "-I" + CSRC,
                        "-mllvm", "-disable-promote-alloca-to-lds", *defines,
                        "--offload-device-only", "-S", "-o", out, src], check=True,
                       stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        return out
    with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        return list(ex.map(one, srcs))


def main(argv):
    if argv:
        files = argv
        tmp = None
    else:
        tmp = tempfile.TemporaryDirectory()
        files = compile_all(tmp.name)
    total = 0
    for f in files:
        for func, line, st, what, rule in scan(f):
            total += 1
            print(f"{os.path.basename(f)}:{line} {func}: [{rule}] {st}  ->  {what}")
    print(f"wide-store hazards: {total} in {len(files)} file(s)")
    return 1 if total else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
