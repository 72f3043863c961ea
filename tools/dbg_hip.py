import ctypes, os, sys
print("env", {k: v for k, v in os.environ.items() if "VISIBLE" in k or "HIP" in k or "ROC" in k or "HSA" in k})
mode = sys.argv[1]
if mode == "torch_first":
    import torch
    print("torch avail", torch.cuda.is_available(), torch.cuda.device_count())
lib = ctypes.CDLL("/opt/rocm/lib/libamdhip64.so.7")
n = ctypes.c_int(-1)
print("hipGetDeviceCount rc", lib.hipGetDeviceCount(ctypes.byref(n)), n.value)
d = ctypes.c_int(-1)
print("hipGetDevice rc", lib.hipGetDevice(ctypes.byref(d)), d.value)
with open("/proc/self/maps") as f:
    print(sorted({l.split()[-1] for l in f if "amdhip" in l or "hsa-runtime" in l}))
if mode == "lib_first":
    import torch
    print("torch avail", torch.cuda.is_available(), torch.cuda.device_count())
    with open("/proc/self/maps") as f:
        print(sorted({l.split()[-1] for l in f if "amdhip" in l or "hsa-runtime" in l}))
