import sys, os, numpy as np
sys.path.insert(0,'tests'); sys.path.insert(0,'sentencepiece-comments_amd')
import oracle_lib as O, spm_amd as S, model_reader
mb=open('tests/golden/test_model.model','rb').read()
pcs=[(p,s) for p,s,t in model_reader.read_pieces(mb) if t==1]
pieces=[p for p,_ in pcs]; scores=np.array([s for _,s in pcs],dtype=np.float32)
lines=O.read_lines_binary('tests/golden/botchan.txt')
allsents=[x for x in O.OracleModel(mb).normalize(lines) if x]
def run(sents, T, mode=S.SPM_ESTEP_PARITY, tag=''):
    freqs=np.arange(len(sents))%5+1
    e_ref,o_ref,n_ref=O.estep(sents,freqs,pieces,scores,T)
    dp=S.DevicePieces(pieces,scores)
    e,o,n=dp.estep(sents,freqs,mode=mode,threads=T)
    nz=e_ref!=0
    print(tag, 'T',T,'n',len(sents),'eq',np.mean(e==e_ref),'maxrel',np.max(np.abs(e-e_ref)[nz]/e_ref[nz]), 'obj',o,o_ref,'ntok',n,n_ref, flush=True)
for k in []:
    run([s for s in allsents if len(s)<=64][:k], 1, tag='short')
for k in []:
    run([s for s in allsents if len(s)>64][:k], 1, tag='long')


base=allsents[:10]
for extra in [[b"a"*300],[b"\xff\xfeabc"],["é".encode()+b"\x80z"],[b"a"*40]]:
    run(base+extra,1,tag='extra%r'%extra[0][:6])
    run(base+extra,1,mode=S.SPM_ESTEP_FAST,tag='extra-fast%r'%extra[0][:6])
