"""Scenario fixtures on disk (YAML + Gmsh MSH 4.1) equivalent to scenarios.block_case(...)."""
import os

from cwf import meshgen

YAML = """mesh:
  path: {msh}
materials:
  - name: steel
    E: 3.0e10
    nu: 0.2
    rho: 2500.0
assignments:
  - group: SOLID
    material: steel
damping:
  xi: {xi}
  w1: {w1}
  w2: {w2}
time:
  dt: 0.01
  adaptive: false
solver:
  type: pcg
  preconditioner: block_jacobi
  tol_runtime: {tol}
  tol_pause: 1.0e-5
  max_iters: {maxit}
precision:
  vectors: fp32
  reductions: fp64
loads:
  gravity: [0.0, 0.0, -9.81]
  points:
    - group: TIP
      value: [0.0, 0.0, -500.0]
dirichlet:
  fixes:
    - group: FIXED
      dof: [x, y, z]
output:
  vtu_stride: {stride}
  probes: [0, 5]
"""


def write_block_scenario(dirname, nx, ny, nz, h=0.1, xi=0.02, w=(5.0, 50.0), tol=3e-4, maxit=2000, stride=2,
                         relative=True, element="tet4"):
    """Writes block.msh + block.yaml for the Kuhn block (same mesh, config and loads as
    scenarios.block_case(nx, ny, nz, h, xi=xi, w=w, tol=tol, max_iterations=maxit)) -> yaml path.
    element="hex8": the same block as native hex8 elements with quad boundary faces."""
    tm = meshgen.hex_block(nx, ny, nz, h) if element == "hex8" else meshgen.kuhn_block(nx, ny, nz, h)
    msh = os.path.join(dirname, "block.msh")
    meshgen.write_gmsh(tm, msh, node_groups=["FIXED", "TIP"])
    y = os.path.join(dirname, "block.yaml")
    with open(y, "w") as f:
        f.write(YAML.format(msh="block.msh" if relative else msh, xi=xi, w1=w[0], w2=w[1], tol=tol, maxit=maxit,
                            stride=stride))
    return y
