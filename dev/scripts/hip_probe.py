"""Which HIP runtime sees the device on the box (diagnostic)."""
import ctypes
import os
import sys

print({k: v for k, v in os.environ.items() if any(s in k for s in ("HIP", "ROCR", "HSA", "GPU", "LD_"))})
first = sys.argv[1] if len(sys.argv) > 1 else "sys"
if first == "torch":
    import torch
    print("torch sees", torch.cuda.device_count())
lib = ctypes.CDLL("/opt/rocm/lib/libamdhip64.so.7")
n = ctypes.c_int(-1)
rv = lib.hipGetDeviceCount(ctypes.byref(n))
print(first, "system hipGetDeviceCount rv", rv, "n", n.value)
s = ctypes.create_string_buffer(256)
lib.hipGetErrorString.restype = ctypes.c_char_p
print(lib.hipGetErrorString(rv))
