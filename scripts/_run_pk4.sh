QHUFF_LIB=nghttp3_amd/lib/libqhuff_stamps.so QHUFF_DECODER=run timeout -k 10 120 python -u scripts/stamp_run3.py
