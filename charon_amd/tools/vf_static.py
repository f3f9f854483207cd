"""Compile charon_amd/tools/vf_probe.hip (k_verify_fused alone) with extra flags and summarize its code object:
per function, instructions, scratch instructions, the highest VGPR / AGPR index; the Miller loop body's scratch
count; the kernel's private segment and VGPR count from the metadata.  A compile-only loop for register-allocation
experiments (no GPU):  python3 charon_amd/tools/vf_static.py [-Dfoo=1 ...] [-mllvm -opt ...]"""
import collections
import os
import re
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
sys.path.insert(0, os.path.dirname(PKG))
from charon_amd import codeobj  # noqa: E402

LLVM = "/opt/rocm/lib/llvm/bin"
DYN = {}
MILLER = [0]


def build(extra, out):
    csrc = os.environ.get("VF_CSRC") or os.path.join(PKG, "csrc")  # a modified copy of the sources (experiments)
    cmd = ["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-I" + csrc,
           "-I" + os.path.join(os.path.dirname(PKG), "include"), "-o", out, os.path.join(HERE, "vf_probe.hip")] + extra
    subprocess.check_call(cmd)


def summarize(lib):
    co = codeobj.code_objects(lib)[0]
    with tempfile.NamedTemporaryFile(suffix=".elf", delete=False) as f:
        f.write(co)
        path = f.name
    dis = subprocess.run([LLVM + "/llvm-objdump", "-d", path], capture_output=True, text=True).stdout
    funcs, cur = collections.OrderedDict(), None
    for ln in dis.split("\n"):
        m = re.match(r"^([0-9a-f]+) <(.+)>:$", ln)
        if m:
            cur = m.group(2)
            funcs[cur] = []
        elif cur and re.match(r"^\s+\S", ln):
            am = re.search(r"//\s*([0-9A-Fa-f]+):", ln)
            funcs[cur].append((int(am.group(1), 16) if am else None,
                               re.sub(r"\s+", " ", ln.split("//")[0]).strip()))
    out = {}
    DYN.clear()
    for name, ins in funcs.items():
        v, a = set(), set()
        for _, l in ins:
            for m in re.finditer(r"\bv\[(\d+):(\d+)\]", l):
                v.update(range(int(m.group(1)), int(m.group(2)) + 1))
            for m in re.finditer(r"\bv(\d+)\b", l):
                v.add(int(m.group(1)))
            for m in re.finditer(r"\ba\[(\d+):(\d+)\]", l):
                a.update(range(int(m.group(1)), int(m.group(2)) + 1))
            for m in re.finditer(r"\ba(\d+)\b", l):
                a.add(int(m.group(1)))
        sc = sum(1 for _, l in ins if l.startswith("scratch_"))
        # loops: backward branches, short (s_branch / s_cbranch_* with a negative simm16) or long (s_getpc_b64,
        # s_add_u32 with a negative offset, ..., s_setpc_b64); the largest loop's body and its scratch instructions
        idx = {ad: k for k, (ad, _) in enumerate(ins) if ad is not None}
        loops = []
        for k, (ad, l) in enumerate(ins):
            m = re.match(r"s_c?branch\w* (\d+)$", l)
            if m and int(m.group(1)) >= 0x8000:
                tgt = ad + 4 + 4 * (int(m.group(1)) - 0x10000)
                if tgt in idx:
                    loops.append((idx[tgt], k))
            if l.startswith("s_getpc_b64") and k + 1 < len(ins):
                m2 = re.match(r"s_add_u32 s\d+, s\d+, (0x[0-9a-f]+)", ins[k + 1][1])
                if m2:
                    off = int(m2.group(1), 16)
                    if off >= 0x80000000:
                        tgt = ad + 4 + off - (1 << 32)
                        if tgt in idx:
                            loops.append((idx[tgt], k))
        big = max(loops, key=lambda x: x[1] - x[0]) if loops else None
        lsc = sum(1 for _, l in ins[big[0]:big[1]] if l.startswith("scratch_")) if big else 0
        out[name] = (len(ins), sc, max(v) if v else -1, max(a) if a else -1, (big[1] - big[0]) if big else 0, lsc)
        # dynamic estimate of scratch instructions per Verify: the innermost (smallest) loop of the Miller loop runs
        # 62 times, cyc_sqr_run's 315 times, the Karabina tail's largest loop 30 times; everything else once
        trips = {"miller_loop_2_l": 62, "cyc_sqr_run": 315, "karabina_l": 30}
        for key, t in trips.items():
            if key in name and loops:
                lp = min(loops, key=lambda x: x[1] - x[0]) if key == "miller_loop_2_l" else big
                inner = sum(1 for _, l in ins[lp[0]:lp[1]] if l.startswith("scratch_"))
                DYN[name] = sc + (t - 1) * inner
        if name not in DYN and loops:
            # the Miller loop inlined into the kernel (op_verify_l_kernel): its doubling iteration is the smallest loop
            # holding ~61 product calls
            ml = [lp for lp in loops if 50 <= sum(1 for _, l in ins[lp[0]:lp[1]] if "swappc" in l) <= 70]
            if ml:
                lp = min(ml, key=lambda x: x[1] - x[0])
                inner = sum(1 for _, l in ins[lp[0]:lp[1]] if l.startswith("scratch_"))
                DYN[name] = sc + 61 * inner
                MILLER[0] = DYN[name]
        DYN.setdefault(name, sc)
        if os.environ.get("VF_LOOPS"):
            for a0, a1 in sorted(set(loops)):
                sub = ins[a0:a1]
                print("   loop in %s: %d ins, %d scratch, %d swappc" % (name[:40], a1 - a0,
                      sum(1 for _, l in sub if l.startswith("scratch_")), sum(1 for _, l in sub if "swappc" in l)))
    res = codeobj.resource_table(lib)
    return out, res


if __name__ == "__main__":
    extra = sys.argv[1:]
    lib = os.path.join(tempfile.gettempdir(), "vf_probe_%d.so" % os.getpid())
    build(extra, lib)
    out, res = summarize(lib)
    for name, (n, sc, mv, ma, ln, lsc) in sorted(out.items(), key=lambda x: -x[1][1])[:12]:
        print("%6d scratch %6d ins  v%-3d a%-3d  loop %5d ins %4d scratch  %s" % (sc, n, mv, ma, ln, lsc, name[:80]))
    for r in res:
        print("kernel", r)
    print("dynamic scratch estimate per Verify: %d (miller %d, karabina %d, cyc_sqr_run %d)" % (
        sum(DYN.values()), sum(v for k, v in DYN.items() if "miller_loop_2_l" in k) or MILLER[0],
        sum(v for k, v in DYN.items() if "karabina_l" in k), sum(v for k, v in DYN.items() if "cyc_sqr_run" in k)))
