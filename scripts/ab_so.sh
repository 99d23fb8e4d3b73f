set -u
mkdir -p /tmp/alt && cp -r tensorframes_amd scripts /tmp/alt/ && cp ab_so/_C_noprio.so /tmp/alt/tensorframes_amd/_C.cpython-310-x86_64-linux-gnu.so || exit 1
for rep in 1 2; do
while read -r sh; do
  timeout -k 5 120 python scripts/gemm_one.py $sh --iters 30 | sed 's/^/PRIO /' || exit 1
  timeout -k 5 120 python /tmp/alt/scripts/gemm_one.py $sh --iters 30 | sed 's/^/BASE /' || exit 1
done < scripts/epi_shapes.txt
done
