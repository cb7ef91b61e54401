set -o pipefail
mkdir -p gpurun_out/r05p
O=gpurun_out/r05p/enc.log
for a in A U; do
for cfg in "0 256" "1 256" "1 128" "0 128"; do set -- $cfg
QHUFF_ENC_SNAKE=$1 QHUFF_ENC_THREADS=$2 QHUFF_VERBOSE=1 timeout -k 10 120 python -u dev/scripts/enc_variants.py --only windows --alphabet $a > gpurun_out/r05p/e_$a$1$2.log 2>&1 || exit 1
echo "snake=$1 nt=$2 $(grep -h 'blocks/CU' gpurun_out/r05p/e_$a$1$2.log | sort -u | tr '\n' ' ') $(tail -1 gpurun_out/r05p/e_$a$1$2.log)" >> $O
done; done
for cfg in "0 256" "1 256" "1 128"; do set -- $cfg
QHUFF_ENC_SNAKE=$1 QHUFF_ENC_THREADS=$2 timeout -k 10 120 python -u dev/scripts/enc_variants.py --only windows --zipf >> $O 2>&1 || exit 1
done
QHUFF_ENC_SNAKE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "enc or round" > gpurun_out/r05p/pytest.log 2>&1 || { tail -20 gpurun_out/r05p/pytest.log; exit 1; }
tail -2 gpurun_out/r05p/pytest.log
cat $O
