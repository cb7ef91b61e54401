set -e
o=gpurun_out/${1:-r06f}
mkdir -p $o
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k region > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -2 $o/pytest.log
timeout -k 10 120 python -u dev/scripts/region_probe.py > $o/base.json 2>&1
QHUFF_LIB=nghttp3_amd/lib/libqhuff_rgs.so timeout -k 10 120 python -u dev/scripts/region_stamps.py > $o/stamps.json 2>&1
for f in nghttp3_amd/lib/libqhuff_rg?*.so; do v=${f#nghttp3_amd/lib/libqhuff_rg}; v=${v%.so}; [ "$v" = s ] && continue; QHUFF_LIB=$f timeout -k 10 120 python -u dev/scripts/region_probe.py > $o/$v.json 2>&1; done
cat $o/*.json | grep -v amdgpu.ids
