"""Offline model of render_pipelined's frame schedule (engine.hip) for the OnRun cadence:
per render, the frame-bounces it traces (x0.8) and shades (x0.2), for injection rules of the
pipeline fill (r06 pacing study).  Units: a lone 1-spp frame of depth D = D.
The model's per-render shape matches the measured OnRun times of profiles/r06_pacing.txt
(e.g. G 2, K = D = 4: fill [4, 4, 10, 4, 3.2, 14.8, 6.4, 1.6] vs measured 2.9, 2.9, 5.8, 1.9,
1.7, 8.1, 3.6, 0.9 ms).  usage: python tools/pipe_schedule_model.py"""
def sim(G, K, D, rule, renders=80):
    pipe=[]; run_=0; half=False; out=[]; depths=[]
    for r in range(renders):
        cont = r > 0; speculate = cont and run_ >= 1
        if not cont: pipe=[]; run_=0
        else: run_ += 1
        st={'w':0.0,'ahead':0,'fresh':False}
        def trace_half(it, L, rn):
            had=bool(pipe); inflight=sum(g['f'] for g in pipe if g['ph']<D)
            if not had: st['fresh']=True
            inject=(not had) or (speculate and len(pipe)<K and it+rn+1>=L)
            if inject and had: inject = rule(st, it, L, inflight, G, D)
            if inject and had: st['ahead']+=1
            w=inflight
            if inject:
                f=G if speculate and had else 1
                pipe.append({'f':f,'ph':0,'c':0}); w+=f
            st['w']+=w
            return 0.8*w
        def shade_half():
            w=sum(g['f'] for g in pipe if g['ph']<D)
            for g in pipe: g['ph']+=1
            return 0.2*w
        work=0.0
        if half: half=False; work+=shade_half()
        L = D if not pipe else D-pipe[0]['ph']
        for it in range(L): work+=trace_half(it,L,run_); work+=shade_half()
        g=pipe[0]; g['c']+=1
        if g['c']==g['f']: pipe.pop(0)
        if G>1 and speculate and L==0 and pipe and pipe[0]['ph']<D:
            work+=trace_half(0,D-pipe[0]['ph'],run_+1); half=True
        out.append(round(work,2)); depths.append(len(pipe))
    st=out[40:]
    return out[:12], max(out[:40]), sum(st)/len(st), max(st), depths[-1]
rules = {
 'none': lambda st,it,L,inf,G,D: True,
 'fresh1': lambda st,it,L,inf,G,D: (not st['fresh']) or st['ahead'] < 1,
 'budget2+last': lambda st,it,L,inf,G,D: it == L-1 or st['w'] + (L-it)*(inf+G) <= 2*D*max(G,1),
 'budget1.5+last': lambda st,it,L,inf,G,D: it == L-1 or st['w'] + (L-it)*(inf+G) <= 1.5*D*max(G,1),
 'fresh1+budget2+last': lambda st,it,L,inf,G,D: ((not st['fresh']) or st['ahead'] < 1) and (it == L-1 or st['w'] + (L-it)*(inf+G) <= 2*D*max(G,1)),
 'ahead2': lambda st,it,L,inf,G,D: st['ahead'] < 2,
 'fresh1+ahead2': lambda st,it,L,inf,G,D: st['ahead'] < (1 if st['fresh'] else 2),
}
for G,K,D in ((2,4,4),(1,4,4),(1,8,8),(2,5,5),(2,8,8),(1,5,5)):
    for name,rule in rules.items():
        first, fmax, smean, smax, dep = sim(G,K,D,rule)
        print(f"G{G} K{K} D{D} {name:22s} fill max {fmax:5.1f} steady mean {smean:4.2f} max {smax:4.1f} groups {dep}  {first}")
