"""The reference's own known answers for the native GJK/EPA solver mjc_ccd
(test/engine/engine_collision_gjk_test.cc, MjGjkTest), restated as data: each case's model,
the geom frames the test overrides after mj_forward, the call (the test file's GeomDist
helper, :62-84, or its Penetration helper, :86-150) and the expected values at the test's
tolerance. Test data only: the expected numbers are the ones that file asserts.

Shared by tests/test_gjk_kat_cpu.py (oracle and the device code compiled for the host) and
tests/test_gjk_kat_gpu.py (mjhip_ccdBatch on the device).

The helpers' config (:43-44, :65-71, :123-131): max_iterations 1000 (kMaxIterations),
tolerance 1e-6 (kTolerance); GeomDist: margin 0, max_contacts 0, dist_cutoff (default
mjMAXVAL); Penetration: object margin `margin` on both geoms, max_contacts 1, dist_cutoff 0,
and the reported contact is dir = normalize(x1 - x2), pos = (x1 + x2) / 2 when dist < 0.
"""
import numpy as np

KTOL = 1e-6            # kTolerance (:43)
KMAX = 1000            # kMaxIterations (:44)
MAXVAL = 1e10          # mjMAXVAL

# kEllipoid (:45-60)
ELLIPSOID = """<mujoco model="Ellipsoid Test">
  <compiler angle="radian"/>
  <size nkey="1"/>
  <worldbody>
    <geom name="geom1" size="0.1 0.1 0.1" pos="0 0 -0.1" type="ellipsoid"/>
    <body pos="0 0 0.1">
      <joint type="free" limited="false"/>
      <geom name="geom2" size="0.01 0.02 0.1" type="ellipsoid"/>
    </body>
  </worldbody>
  <keyframe>
    <key time="1.446"
      qpos="0.000886189 -0.0303047 0.0951303 0.98783 0.155468 0.00454524 1.60038e-06"
      qvel="0.00769267 -0.258656 -0.0775641 2.73712 0.0813998 -0.000166485"/>
  </keyframe>
</mujoco>"""

SPHERES = """<mujoco><worldbody>
  <geom name="geom1" type="sphere" pos="-1.5 0 0" size="1"/>
  <geom name="geom2" type="sphere" pos="1.5 0 0" size="1"/>
</worldbody></mujoco>"""

BOX_MESHES = """<mujoco><asset>
  <mesh name="box" scale=".5 .5 .1" vertex="-1 -1 -1  1 -1 -1  1 1 -1  1 1 1  1 -1 1
        -1 1 -1  -1 1 1  -1 -1 1"/>
  <mesh name="smallbox" scale=".1 .1 .1" vertex="-1 -1 -1  1 -1 -1  1 1 -1  1 1 1  1 -1 1
        -1 1 -1  -1 1 1  -1 -1 1"/></asset>
  <worldbody>
    <geom name="geom2" pos="0 0 .1" size=".1 .1 .1" type="mesh" mesh="smallbox"/>
    <geom name="geom1" pos="0 0 -.099999999" size=".5 .5 .1" type="mesh" mesh="box"/>
  </worldbody></mujoco>"""

ELLIPSOIDS = """<mujoco><worldbody>
  <geom name="geom1" type="ellipsoid" pos="1.5 0 -.5" size=".15 .30 .20"/>
  <geom name="geom2" type="ellipsoid" pos="1.5 .5 .5" size=".10 .10 .15"/>
</worldbody></mujoco>"""

LONG_BOX = """<mujoco><asset>
  <mesh name="long_box" vertex="-1 -1 -1 1 -1 -1 1 1 -1 1 1 1 1 -1 1 -1 1 -1 -1 1 1 -1 -1 1"
        scale=".6 .03 .03"/></asset>
  <worldbody>
    <geom name="geom1" type="box" size="1 1 .3" pos="0 0 -.3"/>
    <geom name="geom2" type="mesh" mesh="long_box" pos="0 0 .02" euler="0 0 40"/>
  </worldbody></mujoco>"""


def _boxes(size1, pos1, size2, pos2):
  return (f'<mujoco><worldbody><geom name="geom1" type="box" pos="{pos1}" size="{size1}"/>'
          f'<geom name="geom2" type="box" pos="{pos2}" size="{size2}"/></worldbody></mujoco>')


# BoxBoxDepth2 (:318-332): geom 1's frame after mj_forward
DEPTH2_FRAMES = {1: ([-0.000171208577507291721461757383, -0.000171208577507290908310128019,
                      1.067119586248553853025100579544],
                     [0.999999966039443077825410455262, -0.000000033960556969622165789148,
                      -0.000260616790777324182967061850, -0.000000033960556972087627235699,
                      0.999999966039443077825410455262, -0.000260616790777321797722282382,
                      0.000260616790777324182967061850, 0.000260616790777321797722282382,
                      0.999999932078886044628518448008])}

# BoxBoxDepth3 (:368-404): both frames
DEPTH3_FRAMES = {0: ([-0.015346499999999199323474918799, -0.023505500000000002086553152481,
                      -4.562296442400120888294168253196],
                     [0.965925826289068201191412299522, -0.258819045102520739476403832668,
                      0.000000000000000006339100926609, 0.258819045102520739476403832668,
                      0.965925826289068201191412299522, -0.000000000000000214827792362716,
                      0.000000000000000049478422780336, 0.000000000000000209148392896446,
                      1.000000000000000000000000000000]),
                 1: ([-0.015346499999999797803074130798, -0.023505499999999998617106200527,
                      -4.659230360891631228525966434972],
                     [0.866025403784438707610604524234, -0.499999999999999944488848768742,
                      0.000000000000000018716705841316, 0.499999999999999944488848768742,
                      0.866025403784438707610604524234, -0.000000000000000263161736875730,
                      0.000000000000000115371725704125, 0.000000000000000237263102359077,
                      1.000000000000000000000000000000])}

# name, model, key (keyframe index or None), frame overrides, call, geoms (by name), kwargs,
# expected. call "dist": GeomDist -> checks on dist (and x1/x2); "pen": Penetration -> checks
# on ncon, dist, dir, pos. Expected entries: ("eq", value) is EXPECT_EQ, ("near", value, tol)
# is EXPECT_NEAR; "x1"/"x2"/"dir"/"pos" take 3-vectors; "abspos0" is |pos[0]|; "if1" applies
# the checks only when ncon == 1 (BoxBoxDepth2's `if (ncons == 1)`).
CASES = [
    ("SphereSphereDist", SPHERES, None, {}, "dist", ("geom1", "geom2"), {},     # :155-181
     {"dist": ("eq", 1.0), "x1": ("eq", [-.5, 0, 0]), "x2": ("eq", [.5, 0, 0])}),
    ("SphereSphereDistCutoff", SPHERES, None, {}, "dist", ("geom1", "geom2"),   # :183-206
     {"cutoff": .999999}, {"dist": ("eq", MAXVAL)}),
    ("SphereSphereNoDist", SPHERES, None, {}, "pen", ("geom1", "geom2"), {},    # :208-233
     {"ncon": ("eq", 0)}),
    ("SphereSphereIntersect",                                                   # :235-274
     SPHERES.replace('pos="-1.5 0 0" size="1"', 'pos="-1 0 0" size="3"')
            .replace('pos="1.5 0 0" size="1"', 'pos="3 0 0" size="3"'),
     None, {}, "pen", ("geom1", "geom2"), {},
     {"ncon": ("eq", 1), "dist": ("near", -2, KTOL), "dir": ("near", [1, 0, 0], KTOL),
      "pos": ("near", [1, 0, 0], KTOL)}),
    ("BoxBoxDepth", _boxes("2.5 2.5 2.5", "-1 0 0", "1 1 1", "1.5 0 0"), None, {},  # :276-308
     "pen", ("geom1", "geom2"), {},
     {"ncon": ("eq", 1), "dist": ("near", -1, KTOL), "dir": ("near", [1, 0, 0], KTOL)}),
    ("BoxBoxDepth2", _boxes("5 5 .1", "0 0 0", "1 1 1", "0 0 0"), None, DEPTH2_FRAMES,  # :310-358
     "pen", ("geom1", "geom2"), {},
     {"if1": True, "dist": ("near", -0.033401579411886845, KTOL),
      "dir": ("near", [0, 0, 1], KTOL)}),
    ("BoxBoxDepth3", _boxes("0.25 0.25 0.05", "0 0 0", "0.25 0.25 0.05", "0 0 0"), None,  # :360-424
     DEPTH3_FRAMES, "pen", ("geom1", "geom2"), {},
     {"ncon": ("eq", 1), "dist": ("near", -0.003066, KTOL), "dir": ("near", [0, 0, -1], KTOL)}),
    ("BoxBoxTouching", _boxes("1 1 1", "0 0 1.859913200000001376466229885409", "1 1 1",  # :426-452
                              "0 2 1.859913200000001376466229885409"), None, {}, "pen",
     ("geom1", "geom2"), {}, {"ncon": ("eq", 0)}),
    ("SmallBoxMesh", BOX_MESHES, None, {}, "pen", ("geom1", "geom2"), {},       # :942-999
     {"ncon": ("eq", 1), "dist": ("near", 0, KTOL), "dir": ("near", [0, 0, 1], KTOL),
      "abspos0": ("near", 0.08333333, KTOL), "pos12": ("near", [0, 0], KTOL)}),
    ("EllipsoidEllipsoidPenetrating", ELLIPSOID, 0, {}, "pen", ("geom1", "geom2"), {},  # :1401-1420
     {"ncon": ("eq", 1), "dist": ("near", -0.00022548856248122027, KTOL)}),
    ("EllipsoidEllipsoid", ELLIPSOIDS, None, {}, "dist", ("geom1", "geom2"), {},  # :1422-1445
     {"dist": ("near", 0.7542, 1e-4)}),
    ("BoxBox", _boxes("1 1 1", "-1.5 .5 0", "1 1 1", "1.5 0 0"), None, {}, "dist",  # :1447-1470
     ("geom1", "geom2"), {}, {"dist": ("eq", 1.0)}),
    ("LongBox", LONG_BOX, None, {}, "pen", ("geom1", "geom2"), {},              # :1472-1516
     {"ncon": ("eq", 1), "dist": ("near", -0.01, KTOL), "dir": ("near", [0, 0, 1], KTOL),
      "pos": ("near", [0, 0, -0.005], KTOL)}),
    ("EllipsoidEllipsoidIntersect", ELLIPSOIDS, None, {}, "pen", ("geom1", "geom2"),  # :1518-1544
     {"margin": 15}, {"ncon": ("eq", 1), "dist": ("near", -14.245732934582151, KTOL)}),
    ("CapsuleCapsule",                                                          # :1546-1569
     """<mujoco><worldbody>
       <geom name="geom1" type="capsule" pos="-.3 .2 -.4" size=".15 .30"/>
       <geom name="geom2" type="capsule" pos=".3 .2 .4" size=".10 .10"/>
     </worldbody></mujoco>""", None, {}, "dist", ("geom1", "geom2"), {},
     {"dist": ("near", 0.4711, 1e-4)}),
]

# CylinderBoxMargin (:1571-1600) is a whole-pipeline case: mj_forward on this model gives one
# contact whose efc_address is negative (its distance lies between margin - gap and margin).
CYLINDER_BOX_MARGIN = """<mujoco>
  <option><flag gravity="disable"/></option>
  <worldbody>
    <body pos="0 0 .265"><freejoint/>
      <geom type="box" size=".05 .05 .05" margin="0.1" gap="0.1"/></body>
    <body mocap="true"><geom name="geom2" type="cylinder" size=".2 .2"/></body>
  </worldbody></mujoco>"""


def frames(m, oracle, key, overrides):
  """geom_xpos [ngeom, 3], geom_xmat [ngeom, 9] after mj_forward (the oracle's kinematics at
  qpos0 or the keyframe), then the test's overrides (geom id -> (pos, mat))."""
  q = m.qpos0 if key is None else m.key_qpos.reshape(-1, m.nq)[key]
  oracle.inverse(q, np.zeros(m.nv), np.zeros(m.nv))
  xpos = oracle.d.geom_xpos.reshape(-1, 3).copy()
  xmat = oracle.d.geom_xmat.reshape(-1, 9).copy()
  for g, (p, r) in overrides.items():
    xpos[g] = p
    xmat[g] = r
  return xpos, xmat


def call_args(call, kw):
  """(margin, max_contacts, cutoff) of the helper the case calls."""
  if call == "dist":
    return 0.0, 0, kw.get("cutoff", MAXVAL)
  return float(kw.get("margin", 0.0)), 1, 0.0


def report(call, dist, nx, x1, x2):
  """What the helper returns: GeomDist -> {dist, x1, x2 (when nx > 0)}; Penetration ->
  {ncon, dist, dir, pos} (engine_collision_gjk_test.cc:77-82, :134-146)."""
  if call == "dist":
    r = {"dist": dist}
    if nx > 0:
      r["x1"], r["x2"] = np.asarray(x1), np.asarray(x2)
    return r
  if not dist < 0:
    return {"ncon": 0}
  d = np.asarray(x1) - np.asarray(x2)
  d = d / np.sqrt(d @ d)
  pos = 0.5 * (np.asarray(x1) + np.asarray(x2))
  return {"ncon": nx, "dist": dist, "dir": d, "pos": pos}


def check(name, expected, got):
  """The case's EXPECT_* lines on a helper report; raises AssertionError naming the case."""
  if expected.get("if1") and got.get("ncon") != 1:
    return
  for k, e in expected.items():
    if k == "if1":
      continue
    if k == "abspos0":
      val = abs(got["pos"][0])
    elif k == "pos12":
      val = got["pos"][1:]
    else:
      assert k in got, f"{name}: helper reported no {k} ({got})"
      val = got[k]
    if e[0] == "eq":
      assert np.array_equal(np.asarray(val, dtype=float), np.asarray(e[1], dtype=float)), \
          f"{name}: {k} = {val}, expected exactly {e[1]}"
    else:
      assert np.all(np.abs(np.asarray(val, dtype=float) - np.asarray(e[1])) <= e[2]), \
          f"{name}: {k} = {val}, expected {e[1]} +- {e[2]}"


# ---- multicontact (max_contacts > 1, the polytope face turned into a contact polygon,
# engine_collision_gjk.c:1460-2193): boxes. The Penetration helper reports every contact:
# ncon = status.nx, dir / pos per contact (dir[0..2] and pos[0..2] are the first one's).

def _frame(pos, mat):
  return (list(pos), list(mat))


MULTI4_FRAMES = {
    0: _frame([-0.015346718925143524800414063236, -0.023500448793229846561336771060,
               -4.859382717259980388746498647379],
              [0.500063246694118501700643264485, -0.865988885078582182330819705385,
               -0.000015036290463686326402846169, 0.865988885208801795201338791230,
               0.500063246603650646271432833601, 0.000009541064416582982810641038,
               -0.000000743359510433135621196039, -0.000017792396065397684211655677,
               0.999999999841438502734547455475]),
    1: _frame([-0.015347749710384111718197708285, -0.023500601273213628239489025873,
               -4.958782854594746325460619118530],
              [0.999999999448633714038692232862, -0.000033207420761195452995305499,
               -0.000000044925527333868828730462, 0.000033207420790006526530903364,
               0.999999999448428988912951353996, 0.000000641458652741046316968134,
               0.000000044904226121706672357864, -0.000000641460144248257277838641,
               0.999999999999794386695839421009])}

MULTI5_FRAMES = {
    0: _frame([-0.015381524498156991936914650410, -0.023527931890396581310342938309,
               -4.559214004409498421921398403356],
              [0.965955045562010394810670277366, -0.258709898141739669252814337597,
               -0.000196358811267032467391333017, 0.258709919231419560592399875532,
               0.965955055634174608591990818240, 0.000090476785846218643442895324,
               0.000166266546411239724218358860, -0.000138196479997660070767120932,
               0.999999976628582865068040064216]),
    1: _frame([-0.015358668590921718474784363195, -0.023542070504611382203430380855,
               -4.659108354876987156956147373421],
              [0.866076536677693908927722077351, -0.499911388413602053581996642606,
               -0.000190658753729162216972170540, 0.499911409912061843741071243130,
               0.866076540935322825021103199106, 0.000086494189368211055798235654,
               0.000121885643632020743577087929, -0.000170223074359586521841353202,
               0.999999978083999430111816764111])}

MULTI6_FRAMES = {
    1: _frame([0.413029898172642018217004533653, 0.190777715293135141649827346555,
               0.100006658017411736993906856696],
              [-0.412617528992808124677083014831, -0.910903939143411389700588642881,
               -0.000887930675351447824816819576, 0.910904370383107120368038067681,
               -0.412617275794986082537718630192, -0.000460143975736545586020798115,
               0.000052771423713213129642884969, -0.000998683403024198425301793947,
               0.999999499923193035932911243435])}

MULTI7_FRAMES = {
    0: _frame([-0.002020740254618143012105280221, -0.022654384848980465422263463893,
               -4.858542902144324493463045655517],
              [0.482851932827058627495375731087, -0.875697459006381406787511423317,
               0.002823341095436950488190008812, 0.875701084072774249555948244961,
               0.482853601927766051815638093103, -0.000102269990141710693382082198,
               -0.001273702846902712276094815635, 0.002521784120391480209927292933,
               0.999996009134990648803409385437]),
    1: _frame([-0.011066235018223425159988870803, -0.023114696036485724711662115283,
               -4.958375812037025376355359185254],
              [0.999985133805306514176436394337, -0.005293845271528460454113496070,
               0.001306663930443651821383665990, 0.005293871114312041943616993223,
               0.999985987232967277194006783247, -0.000016319793417504115210251922,
               -0.001306559226005186893221354794, 0.000023236861241766870316309210,
               0.999999146181155484924829579541])}

MULTI8_FRAMES = {
    0: _frame([-0.015346500000000000765720820084, -0.023505499999999998617106200527,
               -4.859662640000005140450412000064], [1, 0, 0, 0, 1, 0, 0, 0, 1]),
    1: _frame([-0.015346500000000000765720820084, -0.023505499999999998617106200527,
               -4.958574289672835533338002278470],
              [1, 0, 0, 0, 1, -0.000000000000000015361939765351, 0,
               0.000000000000000015361939765351, 1])}

MULTI9_FRAMES = {
    0: _frame([-0.1071400000000000268807198722242901567370,
               -0.1928599999999999758948376893386011943221,
               0.1749951524564917204607183975895168259740],
              [1.0, -0.0000000000000000000000000000000000050579,
               0.0000000000000000001927715439853908006818,
               0.0000000000000000000000000000000000056403, 1.0,
               -0.0000000000000000030208514688407265124010,
               -0.0000000000000000001927715439853908006818,
               0.0000000000000000030208514688407265124010, 1.0]),
    1: _frame([-0.1071400000000000268807198722242901567370,
               -0.1928599999999999758948376893386011943221,
               0.2156259187793853615566774806211469694972],
              [1.0, 0.0000000000000000000000000000000037070001,
               -0.0000000000000000649578747741268744461630,
               0.0000000000000000000000000000000064174485, 1.0,
               0.0000000000000001558617582226398399563910,
               0.0000000000000000649578747741268744461630,
               -0.0000000000000001558617582226398399563910, 1.0])}

MULTI3_FRAMES = {
    1: _frame([-0.941218618591869393696924817050, 2.209729011624415928594089564285,
               1.095456702630382306296041861060],
              [0.999999806540386004805043285160, -0.000014738590672566122784237219,
               0.000621853651764864637230267874, -0.000621853434269146370175218586,
               0.000014756878555191479777952690, 0.999999806540251667819063641218,
               -0.000014747764440060310685981504, -0.999999999782504311873765345808,
               0.000014747710457105431443303178])}

# BoxEdge / BoxEdge2 / MeshEdge's scene (:1170-1206): two free boxes; box3 rotated
BOX_EDGE = """<mujoco>
  <option><flag nativeccd="enable" multiccd="enable"/></option>
  <worldbody>
    <geom type="box" name="box1" size="5 5 .1" pos="0 0 0"/>
    <body pos="0 0 2"><freejoint/><geom type="box" name="box2" size="1 1 1"/></body>
    <body pos="0 0 4.4" euler="0 90 40"><freejoint/><geom type="box" name="box3" size="1 1 1"/></body>
  </worldbody></mujoco>"""

BOX_EDGE2_FRAMES = {
    1: _frame([0.0005578602979296120537716641152314878127,
               0.0098645950089783600300830102014515432529,
               1.1037596929447945903746131079969927668571],
              [0.9999979704374094557906005320546682924032,
               -0.0017789363449516469497385662279498319549,
               -0.0009457835609818190025430140188689165370,
               0.0017817418144636251123996695255868871755,
               0.9999939910254954655854930933855939656496,
               0.0029737701675293876438233020564894104609,
               0.0009404877299599626429629783963548561587,
               -0.0029754492741947335607277658198199787876,
               0.9999951310803708581786963804916013032198]),
    2: _frame([-0.0218119359455731035013492657981259981170,
               0.9828851949225971829093850828940048813820,
               3.0930077345364814789263618877157568931580],
              [0.0006737475542006746490053537002040684456,
               -0.0095603689585630827196816028390458086506,
               0.9999540716500983084102927023195661604404,
               -0.1095658134726250898527410981841967441142,
               0.9939334085756179604231874691322445869446,
               0.0095766296438734854756802405972848646343,
               -0.9939793149670246297233688892447389662266,
               -0.1095672335264066821203243762283818796277,
               -0.0003778293989772788311065632171903416747])}

BOX_EDGE_EDGE = """<mujoco>
  <option><flag nativeccd="enable" multiccd="enable"/></option>
  <worldbody>
    <geom type="box" name="box1" size="5 5 .1" pos="0 0 -.1"/>
    <body pos="-2 0 2.99" euler="0 10 0"><freejoint/><geom type="box" name="box2" size=".15 1 3"/></body>
    <body pos="2 0 2.99" euler="0 -10 0"><freejoint/><geom type="box" name="box3" size=".15 1 3"/></body>
  </worldbody></mujoco>"""

BOX_EDGE_EDGE_FRAMES = {
    1: _frame([-1.3241298058948087756903078116010874509811,
               0.0000000000000000007148993364299687318184,
               2.8141526153588731773425024584867060184479],
              [0.9182779243587342321575306414160877466202,
               -0.0000000000000000000364268564068890756444,
               0.3959364262547898638544552341045346111059,
               -0.0000000000000000000591321577502441383525, 1.0,
               0.0000000000000000002291443915550544102718,
               -0.3959364262547898638544552341045346111059,
               -0.0000000000000000002338308114719865891040,
               0.9182779243587342321575306414160877466202]),
    2: _frame([1.3241298058948089977349127366323955357075,
               -0.0000000000000000008679606505055748997840,
               2.8141526153588731773425024584867060184479],
              [0.9182779243587342321575306414160877466202,
               0.0000000000000000000728398144756416399722,
               -0.3959364262547898638544552341045346111059,
               -0.0000000000000000001674060251593158490713, 1.0,
               -0.0000000000000000002042889652712837518138,
               0.3959364262547898638544552341045346111059,
               0.0000000000000000002538761903338069406631,
               0.9182779243587342321575306414160877466202])}

# (name, model, frame overrides, geoms, max_contacts, expected): "ncon" exact; "dist", "dir"
# (the first contact's) near; "pos" the whole [ncon, 3] list near (Pointwise, in order)
MULTI_CASES = [
    ("BoxBoxMultiCCD", _boxes("1 1 1", "0 0 1.9", "10 10 1", "0 0 0"), {},      # :454-490
     ("geom1", "geom2"), 1000,
     {"ncon": ("eq", 4), "dist": ("near", -.1, KTOL), "dir": ("near", [0, 0, -1], KTOL),
      "pos": ("near", [[-1.0, 1.0, 0.95], [1.0, 1.0, 0.95], [1.0, -1.0, 0.95],
                       [-1.0, -1.0, 0.95]], KTOL)}),
    ("BoxBoxMultiCCD2", _boxes("1 1 1", "9.5 9.5 1.9", "10 10 1", "0 0 0"), {},  # :492-528
     ("geom1", "geom2"), 1000,
     {"ncon": ("eq", 4), "dist": ("near", -.1, KTOL), "dir": ("near", [0, 0, -1], KTOL),
      "pos": ("near", [[8.5, 10.0, 0.95], [10.0, 10.0, 0.95], [10.0, 8.5, 0.95],
                       [8.5, 8.5, 0.95]], KTOL)}),
    ("BoxBoxMultiCCD3", _boxes("5 5 .1", "0 0 0", "1 1 1", "0 0 0"), MULTI3_FRAMES,  # :530-573
     ("geom1", "geom2"), 1000, {"ncon": ("eq", 4)}),
    ("BoxBoxMultiCCD4", _boxes("0.25 0.25 0.05", "0 0 0", "0.25 0.25 0.05", "0 0 0"),  # :575-639
     MULTI4_FRAMES, ("geom1", "geom2"), 1000,
     {"ncon": ("eq", 8), "dist": ("near", -0.00060425119242707459, KTOL),
      "dir": ("near", [0, 0, -1], KTOL)}),
    ("BoxBoxMultiCCD5", _boxes("0.25 0.25 0.05", "0 0 0", "0.25 0.25 0.05", "0 0 0"),  # :641-706
     MULTI5_FRAMES, ("geom1", "geom2"), 1000,
     {"ncon": ("eq", 8), "dist": ("near", -0.0001077858631973211, KTOL),
      "dir": ("near", [0.00019065, -8.6494189274575805e-05, -1], KTOL)}),
    ("BoxBoxMultiCCD6", _boxes(".5 .5 .1", "0 0 -.1", ".1 .1 .1", "0 0 0"), MULTI6_FRAMES,  # :708-755
     ("geom1", "geom2"), 1000,
     {"ncon": ("eq", 5), "dist": ("near", -0.00009843, KTOL),
      "dir": ("near", [-0.0008879306751646528, -0.00046014397575771832, 1], KTOL)}),
    ("BoxBoxMultiCCD7", _boxes(".25 .25 .05", "0 0 0", ".25 .25 .05", "0 0 0"),  # :757-817
     MULTI7_FRAMES, ("geom1", "geom2"), 1000, {"ncon": ("eq", 8)}),
    ("BoxBoxMultiCCD8", _boxes(".25 .25 .05", "0 0 0", ".25 .25 .05", "0 0 0"),  # :819-878
     MULTI8_FRAMES, ("geom1", "geom2"), 1000, {"ncon": ("eq", 4)}),
    ("BoxBoxMultiCCD9", _boxes(".025 .025 .025", "0 0 0", ".025 .025 .025", "0 0 0"),  # :880-940
     MULTI9_FRAMES, ("geom1", "geom2"), 1000, {"ncon": ("eq", 4)}),
    ("BoxEdge", BOX_EDGE, {}, ("box2", "box3"), 4, {"ncon": ("eq", 2)}),      # :1170-1206
    ("BoxEdge2", BOX_EDGE, BOX_EDGE2_FRAMES, ("box2", "box3"), 4,             # :1208-1279
     {"ncon": ("eq", 2)}),
    ("BoxEdgeEdge", BOX_EDGE_EDGE, BOX_EDGE_EDGE_FRAMES, ("box2", "box3"), 4,  # :1281-1351
     {"ncon": ("eq", 2)}),
]


def report_multi(dist, nx, x1, x2):
  """The Penetration helper's report with several contacts (:134-146)."""
  if not dist < 0:
    return {"ncon": 0}
  x1, x2 = np.asarray(x1).reshape(-1, 3), np.asarray(x2).reshape(-1, 3)
  d = x1 - x2
  d = d / np.sqrt((d * d).sum(axis=1))[:, None]
  return {"ncon": nx, "dist": dist, "dir": d[0], "pos": 0.5 * (x1 + x2)}


# ---- multicontact on meshes (the compiler's mesh polygons, mjCMesh::MakePolygons)
PENTAPRISM = """<mesh name="pentaprism"
    vertex="1 0 0 0.309 0.951 0 -0.809 0.588 0 -0.809 -0.588 0 0.309 -0.951 0
            1 0 1 0.309 0.951 1 -0.809 0.588 1 -0.809 -0.588 1 0.309 -0.951 1"
    scale=".2 .2 .1"/>"""
BOX_MESH = ('<mujoco><asset>' + PENTAPRISM + '</asset><worldbody>'
            '<geom name="geom1" type="box" pos="0 0 -.01" size="3 3 .01"/>'
            '<geom name="geom2" pos="0 0 0.157" euler="0 -90 0" type="mesh" mesh="pentaprism"/>'
            '</worldbody></mujoco>')
BOX_MESH2 = ('<mujoco><asset>' + PENTAPRISM + '</asset><worldbody>'
             '<geom name="geom1" type="box" pos="0 0 -.01" size="3 3 .01"/>'
             '<geom name="geom2" pos="0 0 -0.001" type="mesh" mesh="pentaprism"/>'
             '</worldbody></mujoco>')
MESH_MESH = ('<mujoco><asset><mesh name="box" vertex="-1 -1 -1 1 -1 -1 1 1 -1 1 1 1 1 -1 1 '
             '-1 1 -1 -1 1 1 -1 -1 1" scale="1 1 .01"/>' + PENTAPRISM + '</asset><worldbody>'
             '<geom name="geom1" type="mesh" pos="0 0 -0.01" mesh="box"/>'
             '<geom name="geom2" pos="0 0 -0.001" type="mesh" mesh="pentaprism"/>'
             '</worldbody></mujoco>')
MESH_EDGE = """<mujoco>
  <option><flag nativeccd="enable" multiccd="enable"/></option>
  <asset>
    <mesh name="smallbox" vertex="-1 -1 -1  1 -1 -1   1  1 -1 1  1  1  1 -1  1  -1  1 -1
                                  -1  1  1 -1 -1  1"/>
    <mesh name="floor" vertex="-1 -1 -1  1 -1 -1  1  1 -1 1  1  1  1 -1  1 -1  1 -1
                               -1  1  1 -1 -1  1" scale="5 5 1"/>
  </asset>
  <worldbody>
    <geom type="mesh" name="box1" mesh="floor" pos="0 0 0"/>
    <body pos="0 0 2"><freejoint/><geom type="mesh" mesh="smallbox" name="box2"/></body>
    <body pos="0 0 4.4" euler="0 90 40"><freejoint/>
      <geom type="mesh" mesh="smallbox" name="box3"/></body>
  </worldbody></mujoco>"""

# the same shape as MULTI_CASES
MESH_MULTI_CASES = [
    ("BoxMesh", BOX_MESH, {}, ("geom2", "geom1"), 1000, {"ncon": ("eq", 4)}),     # :1001-1032
    ("BoxMesh2", BOX_MESH2, {}, ("geom2", "geom1"), 1000, {"ncon": ("eq", 5)}),   # :1034-1065
    ("BoxMeshPrune", BOX_MESH2, {}, ("geom2", "geom1"), 4, {"ncon": ("eq", 4)}),  # :1067-1098
    ("MeshMesh", MESH_MESH, {}, ("geom1", "geom2"), 1000, {"ncon": ("eq", 5)}),   # :1100-1133
    ("MeshMeshPrune", MESH_MESH, {}, ("geom1", "geom2"), 4, {"ncon": ("eq", 4)}),  # :1135-1168
    ("MeshEdge", MESH_EDGE, {}, ("box2", "box3"), 4, {"ncon": ("eq", 2)}),        # :1353-1399
    ("LongBoxMulti", LONG_BOX, {}, ("geom1", "geom2"), 1000, {"ncon": ("eq", 4)}),  # :1513-1515
]
