import itertools
PIS, PPL, PRW = 1584, 792, 112
G128 = [list(range(0,4))+list(range(12,16))+list(range(20,28)), list(range(4,12))+list(range(16,20))+list(range(28,32))]
G128 += [[x+32 for x in g] for g in G128]
def cost(mapping, pis=PIS):
    tot = 0; worst = 0
    for u in range(7):
        for r in range(6):
            for q in range(3):
                addr = {}
                for l in range(64):
                    col, h = l & 31, l >> 5
                    slot, im = mapping(col)
                    f = min(4*u + slot, 24); y2p, x2p = divmod(f, 5)
                    el = im*pis + y2p*PRW + (2*x2p + h)*8 + (r&1)*PPL + (r>>1)*PRW + 16*q
                    addr[l] = el*2
                for g in G128:
                    slots = {}
                    for l in g:
                        a = addr[l]; slots.setdefault((a//16) % 16, set()).add(a)
                    c = max(len(v) for v in slots.values()); tot += c; worst = max(worst, c)
    return tot / (7*6*3*4), worst
print("current (slot=col>>3, img=col&7):", cost(lambda c: (c >> 3, c & 7)))
print("slot=col&3, img=col>>2:", cost(lambda c: (c & 3, c >> 2)))
best = []
for perm in itertools.permutations(range(5)):
    def m(c, perm=perm):
        bits = [(c >> i) & 1 for i in range(5)]
        b = [bits[perm[i]] for i in range(5)]
        slot = b[0] | (b[1] << 1); im = b[2] | (b[3] << 1) | (b[4] << 2)
        return slot, im
    best.append((cost(m), perm))
best.sort()
print(best[:3])
for pis in range(1584, 1584+64, 8):
    print(pis, cost(lambda c: (c >> 3, c & 7), pis))
