"""How much of the per-sample lane latency of a chain launch's items is set by where they ran (r06): the
items' measured latency per sample, normalised by the median of their pre-pass cost class, grouped by XCD,
CU, SIMD and wave slot (diagnostic timeline column 15, rt_hip.h rt_scene_chain_diag) -- the share of the
variance each grouping explains, the features of the slowest and fastest waves, and the launch's end if
every item had run at its wave's typical speed.
    python scripts/wave_variance.py ROWS.npz"""
import numpy as np, sys
rows = np.load(sys.argv[1])["rows"].astype(np.int64)
t0 = rows[:, 4].min()
start = (rows[:, 4] - t0) / 1e5; end = (rows[:, 5] - t0) / 1e5; dur=end-start
pix, seg, K, wave, recs = rows[:, 0], rows[:, 1], rows[:, 2], rows[:, 3], rows[:, 6]
hw = rows[:,15]
xcc = hw>>28; h=hw&0xffff
wid = h&15; simd=(h>>4)&3; cu=(h>>8)&15; sh=(h>>12)&1; se=(h>>13)&7
print("xcc", np.unique(xcc), "se", np.unique(se), "sh", np.unique(sh), "cu", np.unique(cu), "simd", np.unique(simd), "wave ids", np.unique(wid)[:20])
m = (wave==0)&(rows[:,13]==0)&(recs>20)&(start<3)&(seg>0)&(K>1)  # segments k >= 1 only: their records are all rendered in the launch (segment 0 and unsplit items also count the pre-pass samples they resumed)
sps = rows[:,12]/64.0
lat = dur/np.maximum(recs,1)*1e3
# predicted: median lat in sps bins
bins = np.percentile(sps[m], np.linspace(0,100,21))
b = np.clip(np.digitize(sps, bins)-1,0,19)
med = np.array([np.median(lat[m&(b==i)]) for i in range(20)])
r = lat/med[b]
print("items", m.sum(), "ratio pct", np.percentile(r[m],[1,10,50,90,99]).round(2))
cuid = ((xcc*8+se)*2+sh)*16+cu
def expl(key, name):
    keys = key[m]; rr = np.log(r[m])
    u, inv = np.unique(keys, return_inverse=True)
    gm = np.bincount(inv, weights=rr)/np.bincount(inv)
    var_between = np.var(gm[inv]); var_tot = np.var(rr)
    print(f"{name}: groups {len(u)}, var explained {var_between/var_tot:.3f}, group mean ratio pct {np.exp(np.percentile(gm,[1,10,50,90,99])).round(2)}")
expl(xcc, "XCC")
expl(cuid, "CU")
expl(cuid*4+simd, "SIMD")
expl((cuid*4+simd)*16+wid, "wave slot")
# per wave (sim) : group by cuid,simd,wid and start time bucket (same wave instance)
print("--- per-wave features (first items)")
key = (cuid*4+simd)*16+wid
km = key[m]; u, inv = np.unique(km, return_inverse=True)
cnt = np.bincount(inv)
def gmean(x): return np.bincount(inv, weights=x[m])/cnt
wr = np.exp(gmean(np.log(r)))
wlat = gmean(lat)
fs = gmean(sps); fd = gmean(rows[:,11]/64.0)
fsd = np.sqrt(np.maximum(gmean(sps**2)-fs**2,0))
fk = gmean(K.astype(float)); fseg0 = gmean((seg==0).astype(float))
npx = np.array([len(np.unique(pix[m][inv==i])) for i in range(len(u))]) if len(u)<6000 else None
for name, f in [("mean sps", fs), ("sd sps", fsd), ("mean dps", fd), ("mean K", fk), ("seg0 frac", fseg0), ("lanes", cnt.astype(float))]:
    c = np.corrcoef(f, np.log(wr))[0,1]
    print(f"  corr(log wave ratio, {name}) = {c:.3f}")
if npx is not None:
    print("  corr pixels per wave", np.corrcoef(npx, np.log(wr))[0,1])
# slowest waves
o = np.argsort(-wr)[:10]
for i in o:
    print(f"  slow wave ratio {wr[i]:.2f} lanes {cnt[i]} mean sps {fs[i]:.0f} sd {fsd[i]:.0f} dps {fd[i]:.1f} K {fk[i]:.1f} pixels {npx[i] if npx is not None else '-'} lat {wlat[i]:.0f} us")
o = np.argsort(wr)[:5]
for i in o:
    print(f"  fast wave ratio {wr[i]:.2f} lanes {cnt[i]} mean sps {fs[i]:.0f} sd {fsd[i]:.0f} dps {fd[i]:.1f} K {fk[i]:.1f} pixels {npx[i] if npx is not None else '-'} lat {wlat[i]:.0f} us")
# counterfactual: every item at its wave's typical speed (remove the per-wave factor of the first items' waves)
kall = key
wf = np.ones(len(rows))
idx = np.searchsorted(u, kall)
ok = (idx < len(u)) & (u[np.minimum(idx,len(u)-1)] == kall) & (start < 3)
wf[ok] = wr[idx[ok]]
cf = start + dur / wf
print("measured end", end.max().round(1), "end with waves at typical speed", cf.max().round(1),
      "| only slow waves corrected:", (start + dur/np.maximum(wf,1.0)).max().round(1))
