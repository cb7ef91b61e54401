set -o pipefail
mkdir -p gpurun_out/r05al
for L in libqhuff libqhuff_lb8w12 libqhuff_lb8w15 libqhuff libqhuff_lb8w15; do
QHUFF_LIB=nghttp3_amd/lib/$L.so timeout -k 10 120 python -u dev/scripts/enc_variants.py --only windows --alphabet A > gpurun_out/r05al/$L.log 2>&1 || { tail -3 gpurun_out/r05al/$L.log; exit 1; }
echo "$L $(grep encoder gpurun_out/r05al/$L.log | cut -c60-330)"
done
QHUFF_LIB=nghttp3_amd/lib/libqhuff_lb8w15.so timeout -k 10 120 python -u dev/scripts/enc_variants.py --only windows --alphabet U > gpurun_out/r05al/U15.log 2>&1 || exit 1
echo "U lb8w15 $(grep encoder gpurun_out/r05al/U15.log | cut -c60-330)"
