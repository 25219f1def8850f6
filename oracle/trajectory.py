"""ORACLE -- TEST INFRASTRUCTURE ONLY.  Pure-Python restatement of the node's trajectory normalisation.

Planner::normalizeTrajectory (squirrel_8dof_planner.cpp:1557-1637) with findAngularDistance,
findAngularDistanceSigned and normalizeAngle (squirrel_8dof_planner.cpp:2026-2056), term by term in IEEE double
arithmetic (Python floats), so the product's C implementation (csrc/smp_traj.cpp) must agree bit for bit.
"""
import math

PI = math.pi  # M_PI


def angular_distance(a1, a2):                      # squirrel_8dof_planner.cpp:2026-2033
    dist = math.fabs(a2 - a1)
    return dist if dist <= PI else 2 * PI - dist


def angular_distance_signed(a1, a2):               # squirrel_8dof_planner.cpp:2035-2047
    d = a2 - a1
    if math.fabs(d) <= PI:
        return d
    return -2.0 * PI + d if d > 0.0 else 2.0 * PI + d


def normalize_angle(a):                            # squirrel_8dof_planner.cpp:2049-2055
    if a < -PI:
        return a + 2.0 * PI
    if a > PI:
        return a - 2.0 * PI
    return a


def normalize_trajectory(raw, normalized_pose):
    """-> list of poses, or None where the reference returns without touching its output (1561-1562)."""
    dim = len(normalized_pose)
    if dim < 1 or len(raw) <= 1 or len(raw[0]) != dim:
        return None
    traj = [list(map(float, p)) for p in raw]
    if dim > 2:
        for p in traj:                              # 1564-1572
            if p[2] > PI:
                p[2] -= 2.0 * PI
            elif p[2] < -PI:
                p[2] += 2.0 * PI
    out = [list(traj[0])]
    nxt = 1
    full = dim == 8
    while True:
        pn, pl = traj[nxt], out[-1]
        frac = math.fabs(pn[0] - pl[0]) / normalized_pose[0]
        for i in range(1, dim):
            if full and i == 2:
                f = angular_distance(pn[i], pl[i]) / normalized_pose[i]
            else:
                f = math.fabs(pn[i] - pl[i]) / normalized_pose[i]
            if f > frac:
                frac = f
        if frac < 1.0:
            nxt += 1
            if nxt == len(traj):
                out.append(list(traj[-1]))
                return out
            continue
        counter_max = int(frac) + 1                 # (UInt)frac + 1 before the ceil
        frac = float(math.ceil(frac))
        recip = 1.0 / frac
        last = list(out[-1])
        diff = [angular_distance_signed(last[i], pn[i]) if (full and i == 2) else pn[i] - last[i] for i in range(dim)]
        for c in range(1, counter_max + 1):
            p = list(last)
            for j in range(dim):
                p[j] += float(c) * diff[j] * recip
                if full and j == 2:
                    p[j] = normalize_angle(p[j])
            out.append(p)
        nxt += 1
        if nxt == len(traj):
            return out
