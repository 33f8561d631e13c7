"""Run the dword- and qword-read calibration kernels (scripts/calib/calib_fetch.hip) over
1 GiB (past the 256 MiB Infinity Cache); run under rocprofv3 --pmc FETCH_SIZE
and compare FETCH_SIZE*1024 with the 1 GiB read."""
import ctypes, os, torch
here = os.path.dirname(os.path.abspath(__file__))
L = ctypes.CDLL(os.path.join(here, "calib", "libcalib.so"))
n = 1 << 28
x = torch.ones(n, dtype=torch.float32, device="cuda")
out = torch.zeros(2048 * 4, dtype=torch.float32, device="cuda")
torch.cuda.synchronize()
for _ in range(3):
    assert L.calib_run(ctypes.c_void_p(x.data_ptr()), ctypes.c_long(n), ctypes.c_void_p(out.data_ptr()), 2048) == 0
for _ in range(3):
    assert L.calib_run_qword(ctypes.c_void_p(x.data_ptr()), ctypes.c_long(n), ctypes.c_void_p(out.data_ptr()), 2048) == 0
print("read bytes per dispatch", n * 4, "sum", float(out.sum()))
