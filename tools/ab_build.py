"""Build libkcmc.so from the csrc/ of a git revision (or the working tree) into ab/, for
same-box A/B runs: KCMC_LIB_PATH=ab/<name>.so python tools/match_rates.py ...

    python tools/ab_build.py <name> [<git-rev>]     (no rev: the working tree)
    KCMC_AB_FLAGS="-DKCMC_WARP_SENTINEL" python tools/ab_build.py sentinel   (extra compile flags)
    KCMC_AB_PATCH=tools/ab_patches/knn_grid.py python tools/ab_build.py knn_half  (edit the copy first)
"""
import os
import shutil
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)



def main():
    name = sys.argv[1]
    rev = sys.argv[2] if len(sys.argv) > 2 else None
    pkg = "keypoint-consensus-motion-correction_amd"
    sys.path.insert(0, os.path.join(REPO, pkg))
    import build as B  # the package's build.py (flags, sources)

    tmp = tempfile.mkdtemp()
    try:
        csrc = os.path.join(tmp, pkg, "csrc")
        os.makedirs(csrc)
        os.makedirs(os.path.join(tmp, "include"))
        files = {os.path.join("include", "kcmc.h")}
        files |= {os.path.join(pkg, "csrc", f) for f in os.listdir(os.path.join(REPO, pkg, "csrc"))}
        for f in files:
            dst = os.path.join(tmp, f)
            if rev:
                r = subprocess.run(["git", "show", f"{rev}:{f}"], cwd=REPO, capture_output=True)
                if r.returncode != 0:
                    continue
                open(dst, "wb").write(r.stdout)
            else:
                shutil.copy(os.path.join(REPO, f), dst)
        patch = os.environ.get("KCMC_AB_PATCH")  # a script that edits the copied csrc/ (argv[1]) for this build
        if patch:
            subprocess.run([sys.executable, patch, csrc], check=True)
        srcs = [s for s in B.SOURCES if os.path.exists(os.path.join(csrc, s))]
        flags = [f if not f.startswith("-I") else f"-I{os.path.join(tmp, 'include')}" for f in B.COMMON_FLAGS]
        flags += os.environ.get("KCMC_AB_FLAGS", "").split()  # debug macros only (e.g. -DKCMC_WARP_SENTINEL);
        # the product has no A/B macros any more: variants are edits of the copy (KCMC_AB_PATCH)
        objs = []
        for s in srcs:
            o = os.path.join(tmp, s + ".o")
            subprocess.run([B.hipcc(), *flags, *B.EXTRA_FLAGS.get(s, []), "-c", os.path.join(csrc, s), "-o", o],
                           check=True, capture_output=True)
            objs.append(o)
        os.makedirs(os.path.join(REPO, "ab"), exist_ok=True)
        out = os.path.join(REPO, "ab", f"{name}.so")
        subprocess.run([B.hipcc(), f"--offload-arch={B.OFFLOAD_ARCH}", "-shared", "-fPIC", "-o", out, *objs,
                        "-lpthread"], check=True)
        print(out)
    finally:
        shutil.rmtree(tmp)


if __name__ == "__main__":
    main()
