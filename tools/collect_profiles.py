"""File a tools/profile_round.sh output directory under profiles/ with the commit it was
measured on (the GPU box has no .git, so the sha is taken here: HEAD, which must be the
tree that was sent; a dirty tree is recorded as such).

    python tools/collect_profiles.py gpurun_out/<dir> <tag> [--config c2] [--commit <sha>]

Writes profiles/<tag>_bench_<config>.json (the bench line), <tag>_<config>_kernel_stats.md
(rocprofv3 summary of the same command), <tag>_warp_pmc_<config>.txt and the traffic file
bench.py quotes (profiles/warp_pmc_traffic[_<config>].json)."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
import pmc_summary  # noqa: E402
import prof_summary  # noqa: E402


def commit() -> str:
    sha = subprocess.run(["git", "rev-parse", "HEAD"], cwd=REPO, capture_output=True, text=True).stdout.strip()
    dirty = subprocess.run(["git", "status", "--porcelain", "--untracked-files=no"], cwd=REPO, capture_output=True,
                           text=True).stdout.strip()
    return sha + ("-dirty" if dirty else "")


def main():
    a = sys.argv[1:]
    src, tag = a[0], a[1]
    cfg = a[a.index("--config") + 1] if "--config" in a else "c2"
    # --commit <sha>: the tree the GPU run was sent from, when HEAD has moved on since
    sha = a[a.index("--commit") + 1] if "--commit" in a else commit()
    prof = os.path.join(REPO, "profiles")
    line = open(os.path.join(src, "bench.json")).read().strip().splitlines()[-1]
    d = json.loads(line)
    d["measured_commit"] = sha
    with open(os.path.join(prof, f"{tag}_bench_{cfg}.json"), "w") as f:
        f.write(json.dumps(d) + "\n")
    stats = os.path.join(src, "prof", "run_kernel_stats.csv")
    if os.path.exists(stats):
        import contextlib
        import io

        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            prof_summary.main(stats)
        with open(os.path.join(prof, f"{tag}_{cfg}_kernel_stats.md"), "w") as f:
            f.write(buf.getvalue().replace("# rocprofv3 kernel summary:",
                                           f"# commit {sha}\n\n# rocprofv3 kernel summary:", 1))
    pmc = os.path.join(src, "pmc")
    if os.path.isdir(pmc):
        import contextlib
        import io

        name = "warp_pmc_traffic.json" if cfg == "c2" else f"warp_pmc_traffic_{cfg}.json"
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            pmc_summary.main(pmc, os.path.join(prof, name), sha)
        with open(os.path.join(prof, f"{tag}_warp_pmc_{cfg}.txt"), "w") as f:
            f.write(buf.getvalue())
    print(f"filed {src} as {tag} (commit {sha})")


if __name__ == "__main__":
    main()
