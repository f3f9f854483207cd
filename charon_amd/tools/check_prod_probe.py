"""Check tools/prod_probe's lane results against big-integer Montgomery products.
a <- a*b*R^-1 applied `iters` times; round-1 routine R = 2^384 (canonical), radix-2^29 R = 2^406 (mod p)."""
import sys

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB


def main(path):
    h_in = [((0x9E3779B9 * (i + 1)) & 0xFFFFFFFF) ^ ((i * 7919) & 0xFFFFFFFF) for i in range(64 * 24)]
    for l in range(64):
        h_in[l * 24 + 11] &= 0x0FFFFFFF
        h_in[l * 24 + 23] &= 0x0FFFFFFF
    val = lambda ws: sum(w << (32 * i) for i, w in enumerate(ws))
    lines = open(path).read().split("\n")
    ok = True
    k = 0
    while k < len(lines):
        if not lines[k].startswith("variant"):
            k += 1
            continue
        v, iters = int(lines[k].split()[1]), int(lines[k].split()[3])
        rinv = pow(1 << (384 if v == 0 else 406), -1, P)
        for lane in range(4):
            got = val([int(x, 16) for x in lines[k + 1 + lane].split()])
            a, b = val(h_in[lane * 24:lane * 24 + 12]), val(h_in[lane * 24 + 12:lane * 24 + 24])
            if v == 6:
                for _ in range(iters):
                    a = a * a * rinv % P
            else:
                for _ in range(iters):
                    a = a * b * rinv % P
            good = got % P == a and got < 2 * P
            ok &= good
            print("variant %d lane %d: %s" % (v, lane, "ok" if good else "MISMATCH"))
        k += 5
    print("ALL OK" if ok else "FAILED")
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prod_probe_out.txt"))
