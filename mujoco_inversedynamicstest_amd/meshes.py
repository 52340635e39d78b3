"""Mesh and height-field assets of the MJCF subset: the compiler steps whose results reach the
inverse-dynamics path (mesh_vert / mesh_face / mesh_graph, the mesh frame the geom absorbs, the
mesh volume and inertia box; hfield_size / hfield_data).

Restated from the reference compiler (src/user/user_mesh.cc, src/user/user_objects.cc):

  mjCMesh::Compile :403-622    the order of the steps below
  ApplyTransformations :1344   refpos, refquat, scale on the float vertices
  MakeGraph :1663-1860         the convex-hull graph (qhull "Qt": triangulated facets)
  CopyGraph :1863              faces from the hull when the asset gives none
  Process :1458-1522           face centroid, volume and centre of mass, inertia, principal
                               axes (mjuu_eig3), the equivalent inertia box, then Transform
  ComputeVolume :1275, ComputeInertia :1524, Rotate :1583, Transform :1613
  mjCHField::Compile (user_objects.cc:3696-3783): elevation data normalized to [0, 1]
  xml_native_reader.cc:3286-3293: XML elevation rows are top-to-bottom (stored flipped)

The vertices are float (mjModel.mesh_vert is float), and every step keeps the reference's
float/double mix: float *= double rounds back to float after a double product, the inertia
sums of ComputeInertia are float products of float vertices, and so on.

The hull comes from scipy's Qhull (scipy.spatial.ConvexHull, option Qt) where the reference
links Qhull itself. The graph's content (which hull vertices are adjacent) is the same, but
its ORDER is not pinned: here the vertices are in point-id order and each vertex's edge list
follows its facets in scipy's facet order with the vertices of each facet as scipy lists
them, where the reference walks Qhull's vertex list (FORALLvertices) and each vertex's
neighbour facets (user_mesh.cc:1732-1781). scipy exposes neither list, and neither Qhull's
headers nor its library are in this image, so the reference's order cannot be derived here.
The order is observable in three places:
  * mjc_hillclimbSupport: which support vertex wins a tie (a hull face parallel to the
    search direction);
  * mjc_PlaneConvex (engine_collision_convex.c:1110-1131): after the support vertex it walks
    that vertex's edge list and stops at maxplanemesh = 3 contacts, so when more than two
    neighbours lie within the plane's threshold (a flat face resting on the plane) the order
    picks which two become contacts, and in any case it sets the contacts' order;
  * the face order changes the rounding of the mass-property sums (their last bits).
Plane-mesh contact sets and orders are therefore a known deviation: the oracle compiles from
this module, so tests/test_mesh_hfield_cpu.py pins the device against the oracle, not
against the reference's contact set (Meshes and height fields).
"""
from __future__ import annotations

import math

import numpy as np

mjMINVAL = 1e-15
mjEPS = 1e-14
f32 = np.float32


class MeshError(ValueError):
  pass


def _cross(b, c):
  return [b[1]*c[2] - b[2]*c[1], b[2]*c[0] - b[0]*c[2], b[0]*c[1] - b[1]*c[0]]


def _triangle(v1, v2, v3):
  """_triangle (user_mesh.cc:79-108) on float vertices: (area, normal, center)."""
  # center: (v1 + v2 + v3)/3 with float adds, then the float sum / 3 (int) in float
  cen = [float((f32(v1[i]) + f32(v2[i]) + f32(v3[i])) / f32(3)) for i in range(3)]
  b = [float(f32(v2[i]) - f32(v1[i])) for i in range(3)]     # float difference -> double
  c = [float(f32(v3[i]) - f32(v1[i])) for i in range(3)]
  nrm = _cross(b, c)
  ln = math.sqrt(nrm[0]*nrm[0] + nrm[1]*nrm[1] + nrm[2]*nrm[2])
  if ln < mjMINVAL:
    return 0.0, nrm, cen
  return ln/2, [nrm[0]/ln, nrm[1]/ln, nrm[2]/ln], cen


def _quat2mat(q):
  from .mjcf import quat2mat
  return quat2mat(q)


def hull_graph(vert):
  """MakeGraph (user_mesh.cc:1663-1860): [numvert, numface, vert_edgeadr, vert_globalid,
  edge_localid (per hull vertex its neighbours' local ids, then -1), face_globalid (outward
  triangles)], or None for fewer than 4 vertices."""
  from scipy.spatial import ConvexHull
  n = len(vert)
  if n < 4:
    return None
  pts = np.asarray(vert, dtype=np.float64)
  if not np.isfinite(pts).all():
    raise MeshError("vertex coordinate is not finite")
  try:
    hull = ConvexHull(pts, qhull_options="Qt")
  except Exception as e:             # qhull error (flat or degenerate point set)
    raise MeshError(f"qhull error: {e}") from e
  faces = [list(map(int, s)) for s in hull.simplices]
  # outward orientation (qhull's toporient flip): the normal points away from the hull centre
  ctr = pts[hull.vertices].mean(axis=0)
  for f in faces:
    a, b, c = pts[f[0]], pts[f[1]], pts[f[2]]
    if np.dot(np.cross(b - a, c - a), a - ctr) < 0:
      f[0], f[1] = f[1], f[0]
  gid = sorted(int(v) for v in hull.vertices)
  local = {g: i for i, g in enumerate(gid)}
  numvert, numface = len(gid), len(faces)
  edgeadr, edges = [], []
  for g in gid:
    edgeadr.append(len(edges))
    start = len(edges)
    for f in faces:                   # the vertex's neighbouring facets, facet order
      if g not in f:
        continue
      for v in f:
        if v != g and local[v] not in edges[start:]:
          edges.append(local[v])
    edges.append(-1)
  if len(edges) != numvert + 3*numface:
    raise MeshError("wrong size in convex hull graph")        # SHOULD NOT OCCUR
  return ([numvert, numface] + edgeadr + gid + edges + [v for f in faces for v in f])


def _makenormal(a, b, c):
  """mjuu_makenormal (user_util.cc:362-380) on float vertices: the unit normal of (a, b, c) in
  double (a degenerate triangle keeps the reference's (1, 0, 0) / nrm)."""
  v1 = [float(a[0]), float(a[1]), float(a[2])]
  v2 = [float(b[0]), float(b[1]), float(b[2])]
  v3 = [float(c[0]), float(c[1]), float(c[2])]
  ab = [v2[0]-v1[0], v2[1]-v1[1], v2[2]-v1[2]]
  ac = [v3[0]-v1[0], v3[1]-v1[1], v3[2]-v1[2]]
  n = _cross(ab, ac)
  nrm = math.sqrt(n[0]*n[0] + n[1]*n[1] + n[2]*n[2])
  if nrm < mjEPS:
    n = [1.0, 0.0, 0.0]
  with np.errstate(divide="ignore", invalid="ignore"):
    return [float(np.float64(n[0]) / nrm), float(np.float64(n[1]) / nrm),
            float(np.float64(n[2]) / nrm)]


class _MeshPolygon:
  """MeshPolygon (user_mesh.cc:2058-2269): coplanar faces merged into polygonal sides."""

  def __init__(self, v1, v2, v3, i1, i2, i3):
    self.normal = _makenormal(v1, v2, v3)
    self.edges = [(i1, i2), (i2, i3), (i3, i1)]
    self.islands = [0, 0, 0]
    self.nisland = 1

  def _combine(self, a, b):
    """CombineIslands (:2124-2141): the larger island renumbered into the smaller."""
    if b < a:
      a, b = b, a
    for k in range(len(self.islands)):
      if self.islands[k] == b:
        self.islands[k] = a
      elif self.islands[k] > b:
        self.islands[k] -= 1
    return a, b

  def insert_face(self, v1, v2, v3):
    """InsertFace (:2145-2215)."""
    add = [1, 1, 1]
    island = -1
    for slot, (a, b) in enumerate(((v2, v1), (v3, v2), (v1, v3))):
      for i, e in enumerate(self.edges):
        if e == (a, b):
          other = self.islands[i]
          if slot == 0 or island == -1:
            island = other
          elif other != island:
            self.nisland -= 1
            island, _ = self._combine(island, other)
          add[slot] = 0
          del self.edges[i]
          del self.islands[i]
          break
    if island == -1:
      island = self.nisland
      self.nisland += 1
    for slot, e in enumerate(((v1, v2), (v2, v3), (v3, v1))):
      if add[slot]:
        self.edges.append(e)
        self.islands.append(island)

  def paths(self):
    """Paths (:2218-2269): the vertex cycle of each connected component."""
    E = self.edges
    if len(E) == 3:
      return [[E[0][0], E[1][0], E[2][0]]]
    out = []
    for i in range(self.nisland):
      path = []
      for j in range(len(E)):
        if self.islands[j] == i:
          path = [E[j][0], E[j][1]]
          break
      if not path:
        continue
      nxt = path[-1]
      for _ in range(len(E)):
        finished = False
        for k in range(1, len(E)):        # the reference starts at edge 1
          if self.islands[k] == i and E[k][0] == nxt:
            nxt = E[k][1]
            if nxt == path[0]:
              out.append(path)
              finished = True
              break
            path.append(nxt)
            break
        if finished:
          break
    return out


def _polygon_less(n1, n2):
  """PolygonCmp (user_mesh.cc:2098-2121): the std::set order of the polygons by normal
  (equivalent within the face tolerance, else descending components)."""
  if n1[0]*n2[0] + n1[1]*n2[1] + n1[2]*n2[2] > 0.99999872:
    return False
  for k in range(3):
    if abs(n1[k] - n2[k]) > mjMINVAL:
      return n1[k] > n2[k]
  return False


def make_polygons(vert, faces):
  """mjCMesh::MakePolygons (user_mesh.cc:2272-2330) on the user (unprocessed) float vertices:
  faces of the same plane merged into polygons, kept in a std::set ordered by PolygonCmp
  (restated as a sorted list searched by lower bound), then each polygon's vertex cycles.
  Returns the list of vertex cycles (local vertex ids)."""
  v = np.asarray(vert, dtype=np.float32).reshape(-1, 3)
  polys = []                               # the set, in order
  for f in np.asarray(faces).reshape(-1, 3):
    a, b, c = int(f[0]), int(f[1]), int(f[2])
    face = _MeshPolygon(v[a], v[b], v[c], a, b, c)
    lo, hi = 0, len(polys)
    while lo < hi:                         # lower_bound: first element not less than face
      mid = (lo + hi) // 2
      if _polygon_less(polys[mid].normal, face.normal):
        lo = mid + 1
      else:
        hi = mid
    if lo < len(polys) and not _polygon_less(face.normal, polys[lo].normal):
      polys[lo].insert_face(a, b, c)
    else:
      polys.insert(lo, face)
  return [path for p in polys for path in p.paths() if len(path) >= 3]


class Mesh:
  """One compiled <mesh> asset."""

  def __init__(self, name, vert, face=None, scale=(1, 1, 1), refpos=(0, 0, 0),
               refquat=(1, 0, 0, 0), inertia="legacy", maxhullvert=-1):
    self.name = name
    self.vert = np.asarray(vert, dtype=np.float32).reshape(-1)
    self.face = np.asarray(face if face is not None else [], dtype=np.int64).reshape(-1)
    self.scale = [float(x) for x in scale]
    self.refpos = [float(x) for x in refpos]
    self.refquat = [float(x) for x in refquat]
    self.inertia = inertia
    self.maxhullvert = maxhullvert
    self.needhull = False
    self.graph = None
    self.pos = [0.0, 0.0, 0.0]
    self.quat = [1.0, 0.0, 0.0, 0.0]
    self.aamm = [1e10, 1e10, 1e10, -1e10, -1e10, -1e10]
    self.volume = 0.0
    self.boxsz = [0.0, 0.0, 0.0]
    self.polygons, self.polygon_normals, self.polygon_map = [], [], []

  @property
  def nvert(self):
    return len(self.vert) // 3

  @property
  def nface(self):
    return len(self.face) // 3

  def compile(self, density):
    """mjCMesh::Compile (:403-622), the steps on the path."""
    if len(self.vert) < 12:
      raise MeshError("at least 4 vertices required")
    if len(self.vert) % 3:
      raise MeshError("vertex data must be a multiple of 3")
    if len(self.face) % 3:
      raise MeshError("face data must be a multiple of 3")
    if len(self.face) and (self.face.min() < 0 or self.face.max() >= self.nvert):
      raise MeshError("face vertex index does not exist")
    if self.maxhullvert != -1:
      raise MeshError("maxhullvert is not in the supported subset")
    if self.inertia in ("exact", "shell"):
      raise MeshError(f"mesh inertia '{self.inertia}' is not in the supported subset")
    if self.needhull or not len(self.face):
      self.graph = hull_graph(self.vert.reshape(-1, 3))
    if not len(self.face):                        # CopyGraph
      g = self.graph
      nv, nf = g[0], g[1]
      self.face = np.asarray(g[2 + 3*nv + 3*nf:], dtype=np.int64)
    # MakePolygons (:597) on the graph's faces when there is a graph, before Process
    if self.graph:
      nv, nf = self.graph[0], self.graph[1]
      pfaces = self.graph[2 + 3*nv + 3*nf:]
    else:
      pfaces = self.face
    self.polygons = make_polygons(self.vert, pfaces)
    self._process(density)
    # MakePolygonNormals (:2044-2053) on the processed vertices: the first three of each cycle
    v = self.vert.reshape(-1, 3)
    self.polygon_normals = [_makenormal(v[p[0]], v[p[1]], v[p[2]]) for p in self.polygons]
    # the polygon map (:2320-2326): per vertex, the polygons through it, in order
    self.polygon_map = [[] for _ in range(self.nvert)]
    for i, p in enumerate(self.polygons):
      for vi in p:
        self.polygon_map[vi].append(i)
    return self

  def _apply_transformations(self):
    v = self.vert.reshape(-1, 3)
    rp = [f32(x) for x in self.refpos]
    if any(self.refpos):
      for i in range(len(v)):
        for j in range(3):
          v[i, j] = f32(v[i, j] - rp[j])
    q = self.refquat
    if q[0] != 1 or q[1] != 0 or q[2] != 0 or q[3] != 0:
      from .mjcf import normvec
      qq = list(q)
      normvec(qq)
      mat = _quat2mat(qq)
      for i in range(len(v)):
        p0 = [float(v[i, 0]), float(v[i, 1]), float(v[i, 2])]
        p1 = [mat[0]*p0[0] + mat[3]*p0[1] + mat[6]*p0[2],     # mjuu_mulvecmatT
              mat[1]*p0[0] + mat[4]*p0[1] + mat[7]*p0[2],
              mat[2]*p0[0] + mat[5]*p0[1] + mat[8]*p0[2]]
        v[i] = [f32(p1[0]), f32(p1[1]), f32(p1[2])]
    s = self.scale
    if s[0] != 1 or s[1] != 1 or s[2] != 1:
      for i in range(len(v)):
        for j in range(3):
          v[i, j] = f32(float(v[i, j]) * s[j])

  def _faces(self):
    """The faces the mass properties run over: the hull's for inertia="convex"."""
    if self.inertia == "convex":
      g = self.graph
      nv, nf = g[0], g[1]
      return np.asarray(g[2 + 3*nv + 3*nf:], dtype=np.int64).reshape(-1, 3)
    return self.face.reshape(-1, 3)

  def _process(self, density):
    self._apply_transformations()
    v = self.vert.reshape(-1, 3)
    # ComputeFaceCentroid (:1421-1455)
    facecen = [0.0, 0.0, 0.0]
    area = 0.0
    for f in self.face.reshape(-1, 3):
      a, _, cen = _triangle(v[f[0]], v[f[1]], v[f[2]])
      for j in range(3):
        facecen[j] += a*cen[j]
      area += a
    if area < mjMINVAL:
      raise MeshError(f"mesh volume is too small: {self.name}")
    facecen = [facecen[j] / area for j in range(3)]
    # ComputeVolume (:1275-1311)
    legacy = self.inertia == "legacy"
    faces = self._faces()
    vol_total = 0.0
    com = [0.0, 0.0, 0.0]
    for f in faces:
      a, nrm, cen = _triangle(v[f[0]], v[f[1]], v[f[2]])
      vec = [cen[0]-facecen[0], cen[1]-facecen[1], cen[2]-facecen[2]]
      vol = (vec[0]*nrm[0] + vec[1]*nrm[1] + vec[2]*nrm[2]) * a / 3
      if legacy:
        vol = abs(vol)
      vol_total += vol
      for j in range(3):
        com[j] += vol*(cen[j]*3.0/4.0 + facecen[j]/4.0)
    if vol_total < mjMINVAL:
      raise MeshError(f"mesh volume is {'negative' if vol_total < 0 else 'too small'}: "
                      f"{self.name}")
    com = [com[j] / vol_total for j in range(3)]
    # ComputeInertia (:1524-1580): float vertices centred at the CoM, float products
    vc = np.empty_like(v)
    for i in range(len(v)):
      for j in range(3):
        vc[i, j] = f32(float(v[i, j]) - com[j])
    k = ((0, 0), (1, 1), (2, 2), (0, 1), (0, 2), (1, 2))
    P = [0.0] * 6
    vol_total = 0.0
    for f in faces:
      D, E, F = vc[f[0]], vc[f[1]], vc[f[2]]
      a, nrm, cen = _triangle(D, E, F)
      vol = (cen[0]*nrm[0] + cen[1]*nrm[1] + cen[2]*nrm[2]) * a / 3
      if legacy:
        vol = abs(vol)
      vol_total += vol
      for j in range(6):
        p, q = k[j]
        s = f32(2)*(D[p]*D[q] + E[p]*E[q] + F[p]*F[q]) + D[p]*E[q] + D[q]*E[p] + \
            D[p]*F[q] + D[q]*F[p] + E[p]*F[q] + E[q]*F[p]
        P[j] += density*vol / 20 * float(s)
    self.volume = vol_total
    inert = [P[1] + P[2], P[0] + P[2], P[0] + P[1], -P[3], -P[4], -P[5]]
    from .mjcf import eig3
    full = [inert[0], inert[3], inert[4], inert[3], inert[1], inert[5],
            inert[4], inert[5], inert[2]]
    eigval, quat = eig3(full)
    if eigval[2] <= 0:
      raise MeshError(f"eigenvalue of mesh inertia must be positive: {self.name}")
    atol, rtol = 1e-9, 1e-6
    e = eigval
    if (e[0] + e[1] < e[2]*(1.0 - rtol) - atol or e[0] + e[2] < e[1]*(1.0 - rtol) - atol or
        e[1] + e[2] < e[0]*(1.0 - rtol) - atol):
      raise MeshError(f"eigenvalues of mesh inertia violate A + B >= C: {self.name}")
    mass = self.volume * density
    self.boxsz = [math.sqrt(6*(e[1]+e[2]-e[0])/mass)/2, math.sqrt(6*(e[0]+e[2]-e[1])/mass)/2,
                  math.sqrt(6*(e[0]+e[1]-e[2])/mass)/2]
    # Transform (:1613-1625): CoM to the origin, then Rotate (:1583-1610) by the conjugate
    for i in range(len(v)):
      for j in range(3):
        v[i, j] = f32(float(v[i, j]) - com[j])
    neg = [quat[0], -quat[1], -quat[2], -quat[3]]
    mat = _quat2mat(neg)
    aamm = [1e10, 1e10, 1e10, -1e10, -1e10, -1e10]
    for i in range(len(v)):
      x = [float(v[i, 0]), float(v[i, 1]), float(v[i, 2])]
      res = [mat[0]*x[0] + mat[1]*x[1] + mat[2]*x[2],
             mat[3]*x[0] + mat[4]*x[1] + mat[5]*x[2],
             mat[6]*x[0] + mat[7]*x[1] + mat[8]*x[2]]
      for j in range(3):
        v[i, j] = f32(res[j])
        aamm[j] = min(aamm[j], res[j])
        aamm[j+3] = max(aamm[j+3], res[j])
    self.aamm = aamm
    self.pos = list(com)
    self.quat = list(quat)


class HField:
  """One compiled <hfield> asset (elevation given in the XML)."""

  def __init__(self, name, nrow, ncol, size, elevation):
    self.name = name
    self.nrow, self.ncol = int(nrow), int(ncol)
    self.size = [float(x) for x in size]
    if len(self.size) != 4:
      raise MeshError("hfield size must have 4 values")
    if any(s <= 0 for s in self.size):
      raise MeshError("size parameter is not positive in hfield")
    if self.nrow < 1 or self.ncol < 1 or elevation is None:
      raise MeshError("hfield not specified")
    user = np.asarray(elevation, dtype=np.float32).reshape(-1)
    if user.size != self.nrow*self.ncol:
      raise MeshError("elevation data length must match nrow*ncol")
    data = np.empty_like(user)
    for i in range(self.nrow):                  # top-to-bottom XML rows, stored flipped
      data[(self.nrow - 1 - i)*self.ncol:(self.nrow - i)*self.ncol] = \
          user[i*self.ncol:(i + 1)*self.ncol]
    emin, emax = f32(1e10), f32(-1e10)
    for x in data:
      emin = min(emin, x)
      emax = max(emax, x)
    for i in range(len(data)):
      data[i] = f32(data[i] - emin)
      if emax - emin > mjEPS:
        data[i] = f32(data[i] / (emax - emin))
    self.data = data
