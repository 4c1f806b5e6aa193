# round-5: per-process step-time modes vs translation / L2 counters: the -O2 and -O1 builds, 4 processes each under
# one rocprofv3 pass (UTCL1 translation misses and requests, L2 hits and misses)
set -e
tag=${1:-r05tlb2}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
V=$GRAFT_REPO_ROOT/ti5_isaacgym_amd/_lib/var
for rep in 1 2 3 4; do
  for n in n2b n1b; do
    T1ENV_LIB=$V/libd6_$n.so timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum TCC_HIT_sum TCC_MISS_sum -d $out/${n}_$rep -o p -- python3 $GRAFT_REPO_ROOT/bench.py --steps 200 --warmup 30 --no-cpu-baseline --time-every 0 > $out/${n}_$rep.json 2> $out/${n}_$rep.log
    python3 - <<PY | tee -a $out/summary.txt
import json, sqlite3, glob
d = json.load(open("$out/${n}_$rep.json"))
db = glob.glob("$out/${n}_$rep/**/*.db", recursive=True)[0]
c = sqlite3.connect(db)
q = """select i.name, avg(p.value) from rocpd_pmc_event p join rocpd_info_pmc i on p.pmc_id = i.id
       join rocpd_kernel_dispatch k on k.event_id = p.event_id join rocpd_info_kernel_symbol s on s.id = k.kernel_id
       where s.display_name like '%k_dyn6%' group by i.name"""
vals = {n: v for n, v in c.execute(q)}
print("$n rep $rep", d["ms_per_step"], {k: round(v) for k, v in sorted(vals.items())})
PY
  done
done
