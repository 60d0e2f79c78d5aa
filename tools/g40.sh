# GPU box: raw FETCH_SIZE / WRITE_SIZE of the C2 kernel at 8, 64, 128 and 256 codeblocks per launch (one PMC pass
# each), to split the fetched bytes into a per-CB part (LLRs) and a per-launch part.
cd /root/repo && mkdir -p gpurun_out/fetch && export TMPDIR=/tmp
for n in 8 64 128 256; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d gpurun_out/fetch/${c}_$n -o run -- python3 bench.py --batch $n --steps 10 --warmup 2 --cpu-baseline off --extras off > gpurun_out/fetch/${c}_$n.log 2>&1
    rc=$?; echo "$c n=$n rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
done
python3 - <<'PY'
import collections, csv, glob
for n in (8, 64, 128, 256):
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        v = []
        for f in glob.glob(f"gpurun_out/fetch/{c}_{n}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if "ldpc_decode_kernel" in r["Kernel_Name"] and r["Counter_Name"] == c:
                    v.append(float(r["Counter_Value"]))
        print(f"n={n} {c} KiB avg {sum(v)/max(1,len(v)):.2f} (dispatches {len(v)})")
PY
