"""Build cpp-optical-flow_amd/lab/libhsflow_stamp.so: the library with
per-workgroup s_memrealtime stamps in K2 (hsflow_kernels.hip), for
scripts/lab/stamp_probe.py.  The product sources are copied to a scratch
directory and edited there; the build objects of the other files are
reused (run `make -C cpp-optical-flow_amd` first).
python scripts/lab/make_stamp_lib.py"""
import glob
import os
import shutil
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = os.path.join(ROOT, "cpp-optical-flow_amd")
HIPCC = "/opt/rocm/bin/hipcc"

EDITS = [
    ("namespace hsflow {\n",
     "namespace hsflow {\n__device__ unsigned long long g_stamps[4096][8];\n", 1),
    ("""    asm volatile("; slab parity %0 begin" ::"n"(PAR));""",
     """    asm volatile("; slab parity %0 begin" ::"n"(PAR));
    const int stamp_wg = blockIdx.y * gridDim.x + blockIdx.x;
    auto stamp = [&](int k) {
        const unsigned long long t = __builtin_amdgcn_s_memrealtime();
        if (wv == 2 && lane == 0 && stamp_wg < 4096) g_stamps[stamp_wg][k] = t;
    };
    stamp(0);
    if (wv == 2 && lane == 0 && stamp_wg < 4096)
        g_stamps[stamp_wg][5] = (unsigned long long)tx | ((unsigned long long)ty << 16) |
                                ((unsigned long long)(EDGE ? 1 : 0) << 32) |
                                ((unsigned long long)(ROWE ? 1 : 0) << 33);""", 1),
    ("""    const float inv = p.inv_w2;
    const f2v invv = {inv, inv};""",
     """    stamp(1);
    const float inv = p.inv_w2;
    const f2v invv = {inv, inv};""", 1),
    ("""    int it = 0;
    for (; it + 1 < n_it; ++it) iteration(it, std::false_type{});
    if (it < n_it) iteration(it, std::true_type{});""",
     """    int it = 0;
    for (; it + 1 < n_it; ++it) { iteration(it, std::false_type{}); if (it == 0) stamp(2); }
    if (it < n_it) iteration(it, std::true_type{});
    stamp(3);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    stamp(4);""", 1),
]
EXPORT = """

extern "C" int hsflow_lab_stamps(void *dst) {
    return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(hsflow::g_stamps), sizeof(hsflow::g_stamps), 0,
                                    hipMemcpyDeviceToHost);
}
"""


def main():
    tmp = tempfile.mkdtemp(prefix="hsflow_stamp_")
    for f in glob.glob(os.path.join(PKG, "csrc", "*")):
        shutil.copy(f, tmp)
    src = os.path.join(tmp, "hsflow_kernels.hip")
    s = open(src).read()
    for old, new, n in EDITS:
        assert s.count(old) >= n, old[:60]
        s = s.replace(old, new, n)
    open(src, "w").write(s.rstrip() + EXPORT)
    obj = os.path.join(tmp, "kern_stamp.o")
    subprocess.check_call([HIPCC, "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950",
                           "-fno-slp-vectorize", "-c", src, "-o", obj])
    others = [o for o in glob.glob(os.path.join(PKG, "build", "*.o"))
              if not o.endswith("hsflow_kernels.o")]
    os.makedirs(os.path.join(PKG, "lab"), exist_ok=True)
    subprocess.check_call([HIPCC, "-shared", "--offload-arch=gfx950", "-o",
                           os.path.join(PKG, "lab", "libhsflow_stamp.so"), *others, obj,
                           "-Wl,-rpath,/opt/rocm/lib"])
    shutil.rmtree(tmp)


if __name__ == "__main__":
    main()
