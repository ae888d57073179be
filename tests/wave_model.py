import numpy as np
rng = np.random.default_rng(5)
M = (1<<64)-1
def model_emit_runs(bits):
    # bits: 65536 bool -> words[1024]
    words = [int(x) for x in np.packbits(bits.astype(np.uint8), bitorder='little').view(np.uint64)]
    # lane L holds w[j], j=2k+h : word 128k+2L+h
    W = [[words[128*(j>>1)+2*L+(j&1)] for j in range(16)] for L in range(64)]
    top1 = [sum(((W[L][2*k+1]>>63)&1)<<k for k in range(8)) for L in range(64)]
    bot0 = [sum((W[L][2*k]&1)<<k for k in range(8)) for L in range(64)]
    prev_top = [top1[L-1] if L else ((top1[63]<<1)&0xFE) for L in range(64)]
    next_bot = [bot0[L+1] if L<63 else ((bot0[0]>>1)&0x7F) for L in range(64)]
    def starts(L,j):
        k=j>>1; w=W[L][j]
        prev = (W[L][j-1]>>63) if (j&1) else ((prev_top[L]>>k)&1)
        return w & ~(((w<<1)&M) | prev) & M
    def ends(L,j):
        k=j>>1; w=W[L][j]
        nxt = ((next_bot[L]>>k)&1) if (j&1) else (W[L][j+1]&1)
        return w & ~((w>>1) | (nxt<<63)) & M
    ns = [[bin(starts(L,2*k)).count('1')+bin(starts(L,2*k+1)).count('1') for k in range(8)] for L in range(64)]
    excl = [[sum(ns[l][k] for l in range(L)) for k in range(8)] for L in range(64)]
    tot = [sum(ns[l][k] for l in range(64)) for k in range(8)]
    S = {}; E = {}
    for L in range(64):
        rowoff=0
        for k in range(8):
            sp = rowoff + excl[L][k]; rowoff += tot[k]
            for h in range(2):
                j=2*k+h
                opn = (W[L][j-1]>>63) if h else ((prev_top[L]>>k)&1)
                ep = sp - opn
                base = (128*k+2*L+h)<<6
                x = starts(L,j)
                while x:
                    b=(x&-x).bit_length()-1; S[sp]=base+b; sp+=1; x&=x-1
                y = ends(L,j)
                while y:
                    b=(y&-y).bit_length()-1; E[ep]=base+b; ep+=1; y&=y-1
    r = len(S)
    return [(S[i], E[i]) for i in range(r)]
def true_runs(bits):
    out=[]; x=0
    while x<65536:
        if not bits[x]: x+=1; continue
        s=x
        while x<65536 and bits[x]: x+=1
        out.append((s,x-1))
    return out
for trial in range(20):
    nr = int(rng.integers(1, 2000))
    cuts = np.sort(rng.choice(65537, size=2*nr, replace=False))
    bits = np.zeros(65536, bool)
    for i in range(nr): bits[cuts[2*i]:cuts[2*i+1]] = True
    a = model_emit_runs(bits); b = true_runs(bits)
    print(trial, nr, len(b), a == b)
