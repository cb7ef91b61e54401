set -e
o=gpurun_out/${1:-r06m}; mkdir -p $o
for i in 1 2; do timeout -k 10 150 python -u dev/scripts/host_probe.py 2>&1 | grep '^{' >> $o/host.jsonl; done
cat $o/host.jsonl
