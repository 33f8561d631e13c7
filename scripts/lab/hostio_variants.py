"""Host-I/O lab variants: the product hsflow_hostio.cpp with textual patches,
linked with the product's other objects into cpp-optical-flow_amd/lab/
libhsflow_io_<name>.so (not tracked; travels to the GPU box with the tree).

    python scripts/lab/hostio_variants.py build NAME [NAME ...]   # here
    python scripts/lab/hostio_variants.py probe NAME [NAME ...]   # GPU box

Variants (what sets the tail of hsflow_flow with f64 outputs, main.cpp:98):
  base      the product source unchanged
  spin      the pool threads wait for each landed chunk by polling its event
            (hipEventQuery + pause) instead of hipEventSynchronize
  nofault   no huge-page advice and no prefault (round 4's path)
`probe` runs scripts/pcie/fresh_probe.py with each build in its own process,
alternating the order, and prints the medians per build."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = os.path.join(ROOT, "cpp-optical-flow_amd")
LAB = os.path.join(PKG, "lab")
SRC = os.path.join(PKG, "csrc", "hsflow_hostio.cpp")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-fno-slp-vectorize"]

PATCHES = {
    "base": [],
    "spin": [("        hipError_t e = hipEventSynchronize(events[i]);\n",
              "        hipError_t e;\n"
              "        while ((e = hipEventQuery(events[i])) == hipErrorNotReady) _mm_pause();\n")],
    "nofault": [("    const int nfault = n * kFault;", "    const int nfault = 0 * kFault;"),
                ("    for (int k = 0; k < n; ++k) advise_hugepages(",
                 "    for (int k = 0; k < 0; ++k) advise_hugepages(")],
}


def build(name):
    os.makedirs(LAB, exist_ok=True)
    src = open(SRC).read()
    for old, new in PATCHES[name]:
        assert old in src, (name, old)
        src = src.replace(old, new)
    path = os.path.join(PKG, "csrc", f"_lab_hostio_{name}.cpp")
    with open(path, "w") as f:
        f.write(src)
    obj = os.path.join(LAB, f"hostio_{name}.o")
    try:
        subprocess.check_call(["/opt/rocm/bin/hipcc", *FLAGS, "-c", path, "-o", obj])
    finally:
        os.remove(path)
    objs = [os.path.join(PKG, "build", f) for f in sorted(os.listdir(os.path.join(PKG, "build")))
            if f.endswith(".o") and f != "hsflow_hostio.o"]
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-shared", "--offload-arch=gfx950", "-o",
                           os.path.join(LAB, f"libhsflow_io_{name}.so"), *objs, obj,
                           "-Wl,-rpath,/opt/rocm/lib"])
    print("built", name, flush=True)


def probe(names, rounds=2):
    res = {n: [] for n in names}
    order = (list(names) + list(reversed(names))) * rounds
    script = os.path.join(ROOT, "scripts", "pcie", "fresh_probe.py")
    for n in order:
        env = dict(os.environ, HSFLOW_LIB=os.path.join(LAB, f"libhsflow_io_{n}.so"))
        r = subprocess.run([sys.executable, script, "--reps", "9"], capture_output=True,
                           text=True, timeout=240, env=env)
        line = [x for x in r.stdout.splitlines() if x.startswith("RESULT ")]
        if r.returncode != 0 or not line:
            print(n, "FAILED", r.returncode, r.stderr[-2000:], flush=True)
            return 1
        res[n].append(json.loads(line[0][7:]))
        print(n, line[0][7:], flush=True)
    summary = {}
    for n, runs in res.items():
        summary[n] = {wl: {k: round(sorted(r[wl][k] for r in runs)[len(runs) // 2], 3)
                           for k in ("reused", "fresh", "touched", "huge")}
                      for wl in runs[0]}
    print("SUMMARY " + json.dumps(summary), flush=True)
    return 0


if __name__ == "__main__":
    cmd, names = sys.argv[1], sys.argv[2:]
    if cmd == "build":
        for n in names:
            build(n)
    else:
        sys.exit(probe(names))
