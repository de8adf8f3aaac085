"""Independent symbolic derivation (sympy) of the per-pair d2J_dX2 and d2J_dZdX blocks of the
point-to-point ICP cost J = |R(a,b,c) p + t - q|^2 (R = Rz(a) Ry(b) Rx(c), the reference's
yaw/pitch/roll), evaluated at b = c = z = 0 -- the closed forms of dpg_icp.hip cov6_kernel and
oracle_icp_cov_sandwich (tests/test_cov6.py checks them against the reference's own expressions)."""
import sympy as sp
x, y, z, a, b, c = sp.symbols('x y z a b c', real=True)
px, py, pz, qx, qy, qz = sp.symbols('pix piy piz qix qiy qiz', real=True)
Rz = sp.Matrix([[sp.cos(a), -sp.sin(a), 0], [sp.sin(a), sp.cos(a), 0], [0, 0, 1]])
Ry = sp.Matrix([[sp.cos(b), 0, sp.sin(b)], [0, 1, 0], [-sp.sin(b), 0, sp.cos(b)]])
Rx = sp.Matrix([[1, 0, 0], [0, sp.cos(c), -sp.sin(c)], [0, sp.sin(c), sp.cos(c)]])
R = Rz * Ry * Rx
r = R * sp.Matrix([px, py, pz]) + sp.Matrix([x, y, z]) - sp.Matrix([qx, qy, qz])
J = (r.T * r)[0]
X = [x, y, z, a, b, c]
Z = [px, py, pz, qx, qy, qz]
sub = {b: 0, c: 0, z: 0, pz: 0, qz: 0}
ux, uy = sp.symbols('ux uy', real=True)   # u = R(a) p
rx, ry = sp.symbols('rx ry', real=True)   # r = t + u - q (x, y)
rep = {sp.cos(a) * px - sp.sin(a) * py: ux, sp.sin(a) * px + sp.cos(a) * py: uy}
def simp(e):
    e = sp.expand(sp.simplify(e.subs(sub)))
    return e
H = [[simp(sp.diff(J, X[i], X[j])) for j in range(6)] for i in range(6)]
B = [[simp(sp.diff(J, X[i], Z[j])) for j in range(6)] for i in range(6)]
names = "x y z a b c".split()
zn = "px py pz qx qy qz".split()
for i in range(6):
    for j in range(i, 6):
        print(f"H[{names[i]}{names[j]}] =", sp.factor_terms(H[i][j]))
print()
for i in range(6):
    for j in range(6):
        print(f"B[{names[i]},{zn[j]}] =", sp.factor_terms(B[i][j]))
