# round-5: instruction-cache misses of a fast and a slow k_dyn6 binary (the product build vs the early-read variant,
# 0.125 vs 0.131 ms): one SQC pass per process, 2 processes each
set -e
tag=${1:-r05ic}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
V=$GRAFT_REPO_ROOT/ti5_isaacgym_amd/_lib/var
for rep in 1 2; do
  for n in base se; do
    T1ENV_LIB=$V/libd6_$n.so timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_INSTS_VALU SQ_WAIT_INST_ANY -d $out/${n}_$rep -o p -- python3 $GRAFT_REPO_ROOT/bench.py --steps 100 --warmup 20 --no-cpu-baseline --time-every 0 > $out/${n}_$rep.json 2> $out/${n}_$rep.log
    python3 - <<PY | tee -a $out/summary.txt
import json, sqlite3, glob
db = glob.glob("$out/${n}_$rep/**/*.db", recursive=True)[0]
c = sqlite3.connect(db)
q = """select i.name, avg(p.value) from rocpd_pmc_event p join rocpd_info_pmc i on p.pmc_id = i.id
       join rocpd_kernel_dispatch k on k.event_id = p.event_id join rocpd_info_kernel_symbol s on s.id = k.kernel_id
       where s.display_name like '%k_dyn6%' group by i.name"""
vals = {n: v for n, v in c.execute(q)}
dur = list(c.execute("select avg(d.end - d.start) from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on s.id = d.kernel_id where s.display_name like '%k_dyn6%'"))[0][0]
print("$n rep $rep", round(dur / 1e3, 1), "us", {k: round(v) for k, v in sorted(vals.items())})
PY
  done
done
