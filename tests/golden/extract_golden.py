"""Extract the per-step diag norms from the reference's golden logs into JSON
fixtures.  Run in the build container (needs /root/reference); the JSON it
writes is committed so tests never read /root/reference at run time.

Column slicing follows tests/scripts/test_roms.py:100-103 of the reference:
line[4:26], [27:49], [50:72], [73:95] = KINETIC_ENRG, BAROTR_KE,
MAX_ADV_CFL, MAX_VERT_CFL, printed ES23.16 by diag.F:552.
"""
import json
import os
import sys

REF = "/root/reference/tests"
CASES = {
    "filament_github_gnu": ("Filament/benchmark.result_github_gnu", 20),
    "filament_github_ifx": ("Filament/benchmark.result_github_ifx", 20),
    "pipes_ana_github_gnu": ("Pipes_ana/benchmark.result_github_gnu", 20),
    "pipes_ana_github_ifx": ("Pipes_ana/benchmark.result_github_ifx", 20),
    "rivers_ana_github_gnu": ("Rivers_ana/benchmark.result_github_gnu", 20),
    "rivers_ana_github_ifx": ("Rivers_ana/benchmark.result_github_ifx", 20),
}


def parse(path, ntimes):
    rows = []
    with open(path) as f:
        lines = f.readlines()
    start = None
    for n, line in enumerate(lines):
        if "STEP KINETIC_ENRG" in line:
            start = n + 1
            break
    for line in lines[start:]:
        s = line.rstrip("\n")
        if len(s) < 95 or not s[:2].strip().isdigit():
            continue
        rows.append({"step": int(s[:2]),
                     "ke": s[4:26].strip(), "ke2b": s[27:49].strip(),
                     "cu_adv": s[50:72].strip(), "cu_w": s[73:95].strip()})
        if len(rows) == ntimes + 1:
            break
    return rows


def main():
    out_dir = os.path.dirname(os.path.abspath(__file__))
    for name, (rel, nt) in CASES.items():
        path = os.path.join(REF, rel)
        if not os.path.exists(path):
            print("missing", path, file=sys.stderr)
            continue
        rows = parse(path, nt)
        with open(os.path.join(out_dir, name + ".json"), "w") as f:
            json.dump({"source": "tests/" + rel, "ntimes": nt, "rows": rows}, f, indent=1)
        print(name, len(rows))


if __name__ == "__main__":
    main()
