set -o pipefail
for i in 1 2; do
for v in default oneshot; do
  if [ $v = oneshot ]; then export GM_CHUNK_SUBSTEPS=0; else unset GM_CHUNK_SUBSTEPS; fi
  echo "== $v"
  timeout -k 10 120 python tools/quick_bench_n.py 8 256 20 cylinder 2>&1 | grep "kernel ms" || exit 1
  timeout -k 10 120 python tools/c1_probe.py 2>&1 | grep "rep 1" || exit 1
done
done
