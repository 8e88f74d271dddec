#!/usr/bin/env python3
"""Per-kernel totals and per-split-position times of GBDT tree growth from a rocprofv3 kernel_trace.csv
(usage: prof_tree_breakdown.py <kernel_trace.csv>)."""
import csv, sys, re, collections
def short(n):
    n=n.replace('void ','').replace('sml::(anonymous namespace)::',''); n=re.sub(r'\(.*','',n)
    return n
tot=collections.defaultdict(lambda:[0,0]); 
if sys.argv[1].endswith('.db'):  # rocprofv3's default SQLite output (rocpd schema, `kernels` view)
    import sqlite3
    con = sqlite3.connect(sys.argv[1])
    ks = [(short(n), int(s), int(e), int(l or 0), int(v or 0), int(a or 0), int(sc or 0)) for n, s, e, l, v, a, sc in
          con.execute('select name, start, end, lds_size, vgpr_count, accum_vgpr_count, scratch_size from kernels')]
else:
    rows=list(csv.DictReader(open(sys.argv[1])))
    ks=[(short(r['Kernel_Name']),int(r['Start_Timestamp']),int(r['End_Timestamp']),int(r['LDS_Block_Size']),int(r['VGPR_Count']),int(r['Accum_VGPR_Count']),int(r['Scratch_Size'])) for r in rows]
ks.sort(key=lambda x:x[1])
for n,s,e,*_ in ks: tot[n][0]+=1; tot[n][1]+=e-s
for n,(c,t) in sorted(tot.items(), key=lambda x:-x[1][1]): print(f"{n:40s} {c:6d} {t/1e6:9.2f} ms {t/c/1e3:8.2f} us")
meta={n:(l,v,a,sc) for n,s,e,l,v,a,sc in ks}
for n,m in meta.items(): print(n, 'lds',m[0],'vgpr',m[1],'agpr',m[2],'scratch',m[3])
# per split position within tree: sequence starting at root_init
trees=[]; cur=None
for n,s,e,*_ in ks:
    if n=='root_init_kernel':
        cur=[]; trees.append(cur)
    if cur is not None: cur.append((n,e-s,s,e))
trees=trees[len(trees)//3:]  # the timed fits (bench.py: 1 warm-up + 2 timed fits of 100 trees)
pos=collections.defaultdict(lambda: collections.defaultdict(list))
for t in trees:
    cnt=collections.Counter()
    for n,d,s,e in t:
        pos[n][cnt[n]].append(d); cnt[n]+=1
for n in ('hist_kernel<2>','hist_reduce_kernel','find_split_kernel','choose_part_kernel<8>'):
    print(n, ' '.join(f"{sum(v)/len(v)/1e3:.1f}" for k,v in sorted(pos[n].items())))
# tree wall: root_init start to next root_init start
walls=[]
for t in trees:
    walls.append((t[-1][3]-t[0][2])/1e3)  # includes the gap to the next fit for a fit's last tree
busy=[sum(d for _,d,_,_ in t)/1e3 for t in trees]
print('tree span us avg', sum(walls)/len(walls), 'busy', sum(busy)/len(busy), 'n', len(trees))
gaps=[]; spans=[]
for t in trees:
    g=0
    for i in range(1,len(t)): g+=max(0,t[i][2]-t[i-1][3])
    gaps.append(g/1e3); spans.append((t[-1][3]-t[0][2])/1e3)
print('per tree: span', sum(spans)/len(spans), 'gaps', sum(gaps)/len(gaps), 'kernels', sum(len(t) for t in trees)/len(trees))
import statistics
allg=[]
for t in trees[:-1]:
    for i in range(1,len(t)):
        allg.append((t[i][2]-t[i-1][3])/1e3)
allg.sort()
print('gap count per tree', len(allg)/ (len(trees)-1), 'median', statistics.median(allg), 'p90', allg[int(.9*len(allg))], 'sum<50us per tree', sum(g for g in allg if g<50)/(len(trees)-1))
big=[g for g in allg if g>=50]; print('big gaps', len(big), sum(big)/(len(trees)-1))
# batched speculative growth (round 4): per-round kernel times by round position within the tree
bnames = ('bplan_kernel', 'bpart_kernel', 'bhist_kernel', 'breduce_kernel', 'bfind_kernel')
rpos = collections.defaultdict(lambda: collections.defaultdict(list))
nrounds = []
for t in trees:
    cnt = collections.Counter()
    for n, d, s, e in t:
        for b in bnames:
            if n.startswith(b) or (b == 'bpart_kernel' and n.startswith('bpart_lid_kernel')):
                rpos[b][cnt[b]].append(d)
                cnt[b] += 1
    if cnt['bplan_kernel']:
        nrounds.append(cnt['bplan_kernel'])
if nrounds:
    print('batched growth: plan launches per tree avg %.2f (min %d max %d)' % (sum(nrounds) / len(nrounds), min(nrounds), max(nrounds)))
    print('round  ' + ' '.join(f'{b[:-7]:>9s}' for b in bnames) + '   (us, mean over trees)')
    for r in range(max(nrounds)):
        cells = []
        for b in bnames:
            v = rpos[b].get(r)
            cells.append(f'{sum(v) / len(v) / 1e3:9.1f}' if v else f'{"-":>9s}')
        print(f'{r:5d}  ' + ' '.join(cells))
