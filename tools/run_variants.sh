# Time decoder library variants (make -C srsran_projectvtlmo_amd/csrc exp NAME=...) on the C2 batch.
for v in "$@"; do
  timeout -k 10 120 python tools/time_variant.py srsran_projectvtlmo_amd/lib/libsrsran_ldpc_hip$v.so 2>&1 | grep median || exit 1
done
