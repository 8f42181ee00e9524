"""LDS bank model of csrc/kernels/lenet_band.hip's LDS instructions (lds_sim.py rules,
MI355X_MICROARCH.md § LDS).  Prints worst / mean LDS-array cycles vs the conflict-free
count for each access, over every unit / row / tile position the kernel issues."""
import sys
sys.path.insert(0, __file__.rsplit("/", 1)[0])
import lds_sim as L

L.GROUPS["w_b32"] = [list(range(0, 32)), list(range(32, 64))]
L.NBANK["w_b32"] = 32
L.WIDTH["w_b32"] = 4
L.GROUPS["r2_b64"] = [list(range(16 * i, 16 * i + 16)) for i in range(4)]   # per access
L.NBANK["r2_b64"] = 32
L.WIDTH["r2_b64"] = 8

XRW, XPL, XIS = 32, 448, 900
PRW, PPL, PIS = 112, 792, 1584
XBUF = 8 * XIS


def lanes():
    for lane in range(64):
        col, h = lane & 31, lane >> 5
        yield lane, col, h, col & 1, (col >> 1) & 7, col >> 4


def report(name, kind, addr_sets):
    cs = [L.cycles(kind, a) for a in addr_sets]
    print(f"{name:42s} {kind:7s} worst {max(cs):3d} mean {sum(cs) / len(cs):6.2f} ideal {L.ideal(kind)}")


XZERO = (2 * XBUF + 127) // 128 * 128


def conv1_fetch(split):
    sets = []
    for kb, wave in [(k, w) for k in (0, 1) for w in range(4)]:
        for j in range(14):
            f = min(wave + 4 * j, 48)
            yp0, u = f // 7, f % 7
            for p in range(3):
                S = yp0 + p - 1
                for part in (0, 1):
                    addrs = []
                    for lane, col, h, ypar, img, half in lanes():
                        rlane = 7 * half + ((ypar + h) >> 1)
                        xl = img * XIS + ((ypar + h) & 1) * XPL + rlane * XRW
                        eo = kb * XBUF + xl + S * XRW + 4 * u
                        if 0 <= rlane + S < 14:
                            e = eo
                        elif split == "zrow":
                            e = XZERO + (eo & 127)
                        else:
                            e = 2 * XBUF
                        addrs.append(2 * (e + 4 * part))
                    sets.append(addrs)
    return sets


def conv1_store():
    sets = []
    for wave in range(4):
        for j in range(13):
            f = wave + 4 * j
            if f >= 49:
                continue
            yp0, u = f // 7, f % 7
            addrs = []
            for lane, col, h, ypar, img, half in lanes():
                y = yp0 + 7 * half
                off = (y & 1) * PPL + (y >> 1) * PRW
                addrs.append(2 * (img * PIS + ypar * 8 + 4 * h + off + 16 * u))
            sets.append(addrs)
    return sets


def xfill_store():
    sets = []
    for wave in range(4):
        for i in range(7):
            for part in (0, 1):
                addrs = []
                for lane in range(64):
                    t = 64 * wave + lane
                    r = (t & 31) + 32 * i
                    if r >= 196:
                        addrs.append(None)
                        continue
                    y, k = r // 7, r % 7
                    e = (t >> 5) * XIS + 2 + (y & 1) * XPL + (y >> 1) * XRW + 4 * k
                    addrs.append(2 * e + 4 * part)
                sets.append(addrs)
    return sets


def conv2_read():
    sets = []
    for w2v in range(4):
        for j in range(4):
            f0 = w2v + 4 * j
            if f0 >= 13:
                continue
            for dy in range(5):
                for q in range(3):
                    addrs = []
                    for lane, col, h, ypar, img, half in lanes():
                        fa, fb = f0, min(f0 + 13, 24)
                        ya, yb = fa // 5, fb // 5
                        uoff = yb * PRW + 16 * (fb - 5 * yb) if half else ya * PRW + 16 * (fa - 5 * ya)
                        ce = img * PIS + ypar * PPL + 8 * h
                        co = img * PIS + (1 - ypar) * PPL + ypar * PRW + 8 * h
                        base = (co if dy & 1 else ce) + uoff + (dy >> 1) * PRW
                        addrs.append(2 * (base + 16 * q))
                    sets.append(addrs)
    return sets


def copyout_read():
    sets = []
    NV = 8 * 196
    for e0 in range(0, 256):
        for i in range(4):
            addrs = []
            for lane in range(64):
                t = (e0 // 64) * 64 + lane
                e = min(t + i * 256, NV - 1)
                im, r = e // 196, e % 196
                yp, xp = r // 14, r % 14
                addrs.append(2 * (im * PIS + (yp & 1) * PPL + (yp >> 1) * PRW + xp * 8))
            sets.append(addrs)
        break
    return sets


if __name__ == "__main__":
    report("conv1 fetch as ds_read2_b64 (per access)", "r2_b64", conv1_fetch("one"))
    report("conv1 fetch 2 x ds_read_b64, one zero row", "b64", conv1_fetch("one"))
    report("conv1 fetch 2 x ds_read_b64, bank-matched 0", "b64", conv1_fetch("zrow"))
    report("conv1 epilogue pool1 store ds_write_b64", "w_b64", conv1_store())
    report("input fill ds_write_b32", "w_b32", xfill_store())
    report("conv2 B-fragment ds_read_b128", "b128", conv2_read())
    report("pool1 copy-out ds_read_b128", "b128", copyout_read())
