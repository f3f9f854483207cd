"""Kernel resource metadata of the built library, read from its gfx950 code object (no GPU, no ROCm tools needed).

libhipbls.so carries a clang offload bundle (section .hip_fatbin, magic __CLANG_OFFLOAD_BUNDLE__) whose
`hipv4-amdgcn-amd-amdhsa--gfx950` entry is an AMDGPU ELF code object.  Its NT_AMDGPU_METADATA note (msgpack) lists
every kernel with `.private_segment_fixed_size` (scratch bytes per lane), `.vgpr_count`, `.group_segment_fixed_size`
(LDS) and the rest.

Why it matters: each hardware queue that dispatches a kernel holds a scratch block of the kernel's
private segment x 64 lanes x 32 wave slots per CU x 256 CUs, rounded to 2 MiB (measured: 1,040 B/lane -> 520 MiB,
12,480 B/lane -> 6,240 MiB, profiles/r05/r05_scratch_probe.txt and _layout.txt), and every queue of the process takes
its block from one 32 GiB region per device (HSA_AMD_AGENT_INFO_SCRATCH_LIMIT_MAX), first fit.  A block that grows
leaves a hole, so four queues grown in stages to 12,480 B/lane left no 6.1 GiB gap for a fifth queue: the round-4
abort (HSA_STATUS_ERROR_OUT_OF_RESOURCES).  The library now reserves its four queues' blocks once, contiguously, at
init, so the rest of the region stays one free block.  The budget is what keeps that rest large enough for one more
queue running the library's deepest kernel: (LIBRARY_QUEUES + 1) blocks within the region.  `build.py` refuses a
library whose deepest kernel exceeds it, so a regression fails the build instead of aborting a node under load.
"""
import struct

SCRATCH_REGION = 32 << 30      # HSA_AMD_AGENT_INFO_SCRATCH_LIMIT_MAX on MI355X (profiles/r05/r05_scratch_probe.txt)
WAVE_SLOTS = 64 * 32 * 256     # lanes per wave x scratch wave slots per CU (KFD max_slots_scratch_cu) x CUs
BLOCK_ALIGN = 2 << 20          # blocks are placed on 2 MiB boundaries
LIBRARY_QUEUES = 4             # the library's streams per device (hipbls_device_streams), one hardware queue each
HEADROOM_QUEUES = 1            # queues of the same depth the rest of the region must still hold


def derived_budget(region=SCRATCH_REGION, queues=LIBRARY_QUEUES + HEADROOM_QUEUES):
    """Largest private segment (bytes per lane, a multiple of 16) whose 2 MiB-aligned block fits `queues` times."""
    block = region // queues // BLOCK_ALIGN * BLOCK_ALIGN
    return block // WAVE_SLOTS // 16 * 16


# Bytes of scratch per lane that any kernel may use: 13,104 B (the deepest at the end of round 4: k_rlcb_chunks,
# 12,480 B).  The reserve kernels (k_scratch_reserve<S>) stop at the same figure.
PRIVATE_SEGMENT_BUDGET = derived_budget()
BUNDLE_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
NT_AMDGPU_METADATA = 32


def code_objects(path: str, target: str = TARGET):
    """The code objects of `target` inside the library's offload bundles (one per translation unit: hipbls.hip and
    the eight-lane latency path verify_lat.hip)."""
    with open(path, "rb") as f:
        d = f.read()
    out = []
    i = d.find(BUNDLE_MAGIC)
    while i >= 0:
        (n,) = struct.unpack_from("<Q", d, i + 24)
        p = i + 32
        for _ in range(n):
            off, size, idlen = struct.unpack_from("<QQQ", d, p)
            tid = d[p + 24:p + 24 + idlen].decode()
            p += 24 + idlen
            if tid == target:
                out.append(d[i + off:i + off + size])
        i = d.find(BUNDLE_MAGIC, i + 32)
    if not out:
        raise ValueError("%s: no clang offload bundle with a %s code object (compressed bundles are not expected "
                         "here)" % (path, target))
    return out


def code_object(path: str, target: str = TARGET) -> bytes:
    """The first code object of `target` (the main translation unit's)."""
    return code_objects(path, target)[0]


def _notes(elf: bytes):
    """(name, type, desc) of every note in the ELF64 little-endian image's SHT_NOTE sections."""
    if elf[:4] != b"\x7fELF" or elf[4] != 2 or elf[5] != 1:
        raise ValueError("not an ELF64 little-endian code object")
    shoff, = struct.unpack_from("<Q", elf, 0x28)
    shentsize, shnum = struct.unpack_from("<HH", elf, 0x3A)
    for k in range(shnum):
        sh = shoff + k * shentsize
        sh_type, = struct.unpack_from("<I", elf, sh + 4)
        if sh_type != 7:  # SHT_NOTE
            continue
        off, size = struct.unpack_from("<QQ", elf, sh + 0x18)
        p, end = off, off + size
        while p + 12 <= end:
            namesz, descsz, ntype = struct.unpack_from("<III", elf, p)
            p += 12
            name = elf[p:p + namesz].rstrip(b"\0").decode()
            p += (namesz + 3) & ~3
            desc = elf[p:p + descsz]
            p += (descsz + 3) & ~3
            yield name, ntype, desc


def kernels(path: str):
    """{kernel symbol name: metadata dict} over every gfx950 code object of the library."""
    import msgpack
    out = {}
    for co in code_objects(path):
        found = False
        for name, ntype, desc in _notes(co):
            if name == "AMDGPU" and ntype == NT_AMDGPU_METADATA:
                md = msgpack.unpackb(desc, raw=False)
                out.update({k[".name"]: k for k in md["amdhsa.kernels"]})
                found = True
        if not found:
            raise ValueError("%s: a code object without an AMDGPU metadata note" % path)
    return out


def short_name(mangled: str) -> str:
    """The last component of a nested name: k_verify_fused from _ZN12_GLOBAL__N_114k_verify_fusedEPKh...
    (anonymous-namespace kernels), k_verify_pair_lq8 from _ZN8bls_fp2p17k_verify_pair_lq8EPKjmPi."""
    if not mangled.startswith("_ZN"):
        return mangled
    s, last = mangled[3:], None
    while s and s[0].isdigit():
        j = 0
        while j < len(s) and s[j].isdigit():
            j += 1
        k = int(s[:j])
        last, s = s[j:j + k], s[j + k:]
    return last or mangled


def resource_table(path: str):
    """[(kernel, scratch B/lane, VGPRs incl. AGPRs, LDS B)] sorted by scratch, deepest first."""
    rows = [(short_name(n), int(k.get(".private_segment_fixed_size", 0)), int(k.get(".vgpr_count", 0)),
             int(k.get(".group_segment_fixed_size", 0))) for n, k in kernels(path).items()]
    return sorted(rows, key=lambda r: -r[1])


def check_budget(path: str, budget: int = PRIVATE_SEGMENT_BUDGET):
    """Raises if any kernel's private segment exceeds the budget; returns the resource table otherwise."""
    rows = resource_table(path)
    over = [r for r in rows if r[1] > budget]
    if over:
        raise RuntimeError("kernel private segment above the %d B/lane budget (DESIGN.md 5.1.1): %s"
                           % (budget, ", ".join("%s %d B" % (r[0], r[1]) for r in over)))
    return rows


if __name__ == "__main__":
    import os
    import sys
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                              "libhipbls.so")
    for r in resource_table(lib):
        print("%-28s scratch %6d B/lane  vgpr %4d  lds %6d B" % r)
