QHUFF_LIB=nghttp3_amd/lib/libqhuff_stamps.so KERNELS=enc_lens timeout -k 10 120 python -u scripts/stamp_run.py
