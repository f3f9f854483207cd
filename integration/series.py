"""Maintain the patch series against the reference tree as real files.

    python integration/series.py apply [DIR]   # copy the touched reference files to DIR (default integration/_work)
                                               # and apply 0001..NNNN in order
    python integration/series.py regen [DIR]   # rewrite every patch from DIR: `diff -u` of each file the patch
                                               # touches against /root/reference (new files from integration/charon)

Edit the Go files under DIR, then regen: the patches stay unified diffs of whole edited files, never hand-edited
hunks (a hand-edited hunk once put top-level functions inside `type Implementation interface {`).
A new file in a patch is the file under integration/charon/ (test_new_files_match_integration_tree keeps the two
equal). A new patch is added by creating it with one `--- a/<path>` / `+++ b/<path>` header per file and running regen.
"""
import os
import re
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
PATCHES = os.path.join(HERE, "patches")
CHARON = os.path.join(HERE, "charon")


def series():
    return sorted(os.path.join(PATCHES, f) for f in os.listdir(PATCHES) if f.endswith(".patch"))


def files_of(patch):
    return re.findall(r"^\+\+\+ b/(\S+)", open(patch).read(), flags=re.M)


def apply(work):
    if os.path.exists(work):
        shutil.rmtree(work)
    for p in series():
        for f in files_of(p):
            src = os.path.join(REF, f)
            if os.path.exists(src) and not os.path.exists(os.path.join(work, f)):
                os.makedirs(os.path.dirname(os.path.join(work, f)), exist_ok=True)
                shutil.copy(src, os.path.join(work, f))
    for p in series():
        subprocess.check_call(["patch", "-p1", "--forward", "-s", "-d", work, "-i", p])
    return work


def _diff(a, b, la, lb):
    r = subprocess.run(["diff", "-u", "--label", la, "--label", lb, a, b], capture_output=True, text=True)
    if r.returncode not in (0, 1):
        raise RuntimeError(r.stderr)
    return r.stdout


def regen(work):
    for p in series():
        out = []
        for f in files_of(p):
            ref = os.path.join(REF, f)
            if os.path.exists(ref):
                d = _diff(ref, os.path.join(work, f), "a/" + f, "b/" + f)
            else:
                d = _diff("/dev/null", os.path.join(CHARON, f), "/dev/null", "b/" + f)
            if not d:
                raise SystemExit("%s: %s is unchanged" % (os.path.basename(p), f))
            out.append(d)
        with open(p, "w") as fh:
            fh.write("".join(out))


if __name__ == "__main__":
    cmd = sys.argv[1] if len(sys.argv) > 1 else "apply"
    work = sys.argv[2] if len(sys.argv) > 2 else os.path.join(HERE, "_work")
    {"apply": apply, "regen": regen}[cmd](work)
