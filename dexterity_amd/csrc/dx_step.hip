// dx_step.hip -- the batched physics step for CDNA4 (gfx950).
//
// One 64-thread workgroup (= one wavefront) per environment; the full substep
// pipeline of MuJoCo's mj_step (Euler) runs fused in one launch with all per-env
// state in LDS:
//
//   kinematics (level-parallel over the body tree) -> com / cinert / cdof
//   -> tendon + transmission lengths -> CRB mass matrix
//   -> collision: body-sphere cull (lanes over body pairs) -> geom-sphere cull
//      -> narrowphase one pair per lane (MPR / plane-box / plane-convex / capsules)
//   -> constraint rows (dof friction, joint/tendon limits, pyramidal contacts)
//   -> comVel, RNE + applied wrench, passive, actuation, M^-1 via wave Cholesky
//   -> Newton solver on the primal problem (wave-parallel Hessian, Cholesky,
//      exact line search)
//   -> implicit-damping Euler.
//
// The restated MuJoCo semantics, and where the reference configures each stage,
// are listed in oracle/dx_oracle.c (the fp64 CPU oracle these kernels are
// parity-tested against) and DESIGN.md §3.
#include "dx_device.h"
#include "dx_task.h"
#include <utility>

// 16-byte write-through (sc1) store into a per-env block whose base is wave-uniform:
// the substep queue hands these bytes to the env's next task without a release fence
// (MI355X guide, Guideline 16 R1: sc1 payload, vmcnt(0), flag; the consumer acquires).
typedef unsigned int dx_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st_sc1_f4(void* base, int nbytes, int off, float4 v) {
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(base, 0, nbytes, 0x00020000);
  dx_u32x4 d = {__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)};
  __builtin_amdgcn_raw_buffer_store_b128(d, rsrc, off, 0, 16);
}

// ------------------------------------------------------------------------ //
// collision
// ------------------------------------------------------------------------ //
struct Shape {
  int type, nvert;
  int bin_n, bin_cap;  // direction-binned hull (bin_n > 0), see dx_api.hip build_hull_bins
  float pos[3], mat[9], size[3], center[3], margin;
  const DXG float4* vert4;  // hull vertices (x, y, z, index) in global memory (L2-resident)
  const DXG float4* bin4;   // this hull's cells
};

template <class Ctx>
__device__ __forceinline__ void geom_pose(const Ctx& c, int g, float* pos, float* mat) {
  const DevModel& m = c.mdl();
  int b = m.geom_bodyid[g];
  const float* xp = c.f(c.L.xpos) + 3 * b;
  const float* xm = c.f(c.L.xmat) + 9 * b;
  float t[3];
  matvec3(t, xm, m.geom_pos + 3 * g);
  pos[0] = xp[0] + t[0]; pos[1] = xp[1] + t[1]; pos[2] = xp[2] + t[2];
  matmul3(mat, xm, m.geom_mat + 9 * g);
}

template <class Ctx>
__device__ __forceinline__ void make_shape(const Ctx& c, int g, float half_margin, Shape& s) {
  const DevModel& m = c.mdl();
  s.type = m.geom_type[g];
  geom_pose(c, g, s.pos, s.mat);
  s.size[0] = m.geom_size[3 * g]; s.size[1] = m.geom_size[3 * g + 1]; s.size[2] = m.geom_size[3 * g + 2];
  s.vert4 = m.mesh_vert4;
  s.bin4 = m.mesh_bin4;
  s.nvert = 0;
  s.bin_n = 0;
  s.bin_cap = 0;
  if (s.type == DXG_MESH) {
    int mid = m.geom_dataid[g];
    s.vert4 = m.mesh_vert4 + m.mesh_vertadr[mid];
    s.nvert = m.mesh_vertnum[mid];
    s.bin_n = m.mesh_binn[mid];
    s.bin_cap = m.mesh_bincap[mid];
    s.bin4 = m.mesh_bin4 + m.mesh_binadr[mid];
  }
  float t[3];
  matvec3(t, s.mat, m.geom_center + 3 * g);
  s.center[0] = s.pos[0] + t[0]; s.center[1] = s.pos[1] + t[1]; s.center[2] = s.pos[2] + t[2];
  s.margin = half_margin;
}

struct MPoint { float v[3], a[3], b[3]; };
// dst = c ? src : dst, as value selects (a conditional struct copy lets the optimizer
// merge the copies into one with a selected destination pointer, which pins the
// points in scratch memory).
__device__ __forceinline__ void msel(MPoint& dst, const MPoint& src, bool c) {
#pragma unroll
  for (int k = 0; k < 3; k++) {
    dst.v[k] = c ? src.v[k] : dst.v[k];
    dst.a[k] = c ? src.a[k] : dst.a[k];
    dst.b[k] = c ? src.b[k] : dst.b[k];
  }
}

// MPR's zero test: the oracle's (dx_oracle.c is_zero, |x| < 1e-14), absolute as there.
// (A looser 1e-10 made the degenerate-portal test |v0 x v1|^2 ~ 0 fire for centimetre-scale
// Minkowski vectors up to ~1.4 degrees apart: the "origin on segment v0-v1" shortcut then
// reported a contact whose depth and normal are not a face of the Minkowski difference --
// found on deep finger-finger contacts of the bench's state mix, tools/full_batch_diag.py.)
__device__ __forceinline__ bool fzero(float x) { return fabsf(x) < 1e-14f; }
// The portal points are four separate MPoint variables (not an array): an array of
// structs with conditional element copies stayed an alloca in scratch memory.
__device__ __forceinline__ void portal_dir(const MPoint& P1, const MPoint& P2, const MPoint& P3, float* dir) {
  float a[3], b[3];
  sub3(a, P2.v, P1.v);
  sub3(b, P3.v, P1.v);
  cross3(dir, a, b);
  normalize3(dir);
}
__device__ __forceinline__ bool portal_reach_tol(const MPoint& P1, const MPoint& P2, const MPoint& P3,
                                                 const MPoint& v4, const float* dir, float tol) {
  float dv4 = dot3(v4.v, dir);
  float d1 = dv4 - dot3(P1.v, dir), d2 = dv4 - dot3(P2.v, dir), d3 = dv4 - dot3(P3.v, dir);
  return fminf(d1, fminf(d2, d3)) <= tol;
}
__device__ __forceinline__ void expand_portal(const MPoint& P0, MPoint& P1, MPoint& P2, MPoint& P3,
                                              const MPoint& v4) {
  float v4v0[3];
  cross3(v4v0, v4.v, P0.v);
  bool c1 = dot3(P1.v, v4v0) > 0, c2 = dot3(P2.v, v4v0) > 0, c3 = dot3(P3.v, v4v0) > 0;
  bool to1 = c1 ? c2 : !c3, to2 = !c1 && c3, to3 = c1 && !c2;
  msel(P1, v4, to1);
  msel(P2, v4, to2);
  msel(P3, v4, to3);
}
// Closest point q of triangle abc to the origin and its squared distance (Ericson 5.1.5,
// the oracle's tri_point_dist2), computed in T.  MPR's final portal at a deep overlap
// can be a sliver whose Voronoi-region tests (d1 d4 - d3 d2, ...) cancel in fp32 and pick
// an edge or vertex over the face: a wrong normal and a depth past the closest point
// (bimanual finger-finger contacts at 2-6 mm, test_bimanual_full_batch_parity).  The
// exit runs once per penetrating pair, so it runs in fp64.
template <class T>
__device__ __forceinline__ float tri_origin_dist2_t(const float* af, const float* bf, const float* cf, float* qf) {
  const T a[3] = {af[0], af[1], af[2]}, b[3] = {bf[0], bf[1], bf[2]}, c[3] = {cf[0], cf[1], cf[2]};
  T q[3];
  const T ab[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]}, ac[3] = {c[0] - a[0], c[1] - a[1], c[2] - a[2]};
  auto dot = [](const T* x, const T* y) { return x[0] * y[0] + x[1] * y[1] + x[2] * y[2]; };
  const T ap[3] = {-a[0], -a[1], -a[2]}, bp[3] = {-b[0], -b[1], -b[2]}, cp[3] = {-c[0], -c[1], -c[2]};
  const T d1 = dot(ab, ap), d2 = dot(ac, ap);
  const T d3 = dot(ab, bp), d4 = dot(ac, bp);
  const T d5 = dot(ab, cp), d6 = dot(ac, cp);
  const T vc = d1 * d4 - d3 * d2, vb = d5 * d2 - d1 * d6, va = d3 * d6 - d5 * d4;
  if (d1 <= 0 && d2 <= 0) {
    q[0] = a[0]; q[1] = a[1]; q[2] = a[2];
  } else if (d3 >= 0 && d4 <= d3) {
    q[0] = b[0]; q[1] = b[1]; q[2] = b[2];
  } else if (vc <= 0 && d1 >= 0 && d3 <= 0) {
    const T v = d1 / (d1 - d3);
    for (int k = 0; k < 3; k++) q[k] = a[k] + v * ab[k];
  } else if (d6 >= 0 && d5 <= d6) {
    q[0] = c[0]; q[1] = c[1]; q[2] = c[2];
  } else if (vb <= 0 && d2 >= 0 && d6 <= 0) {
    const T w = d2 / (d2 - d6);
    for (int k = 0; k < 3; k++) q[k] = a[k] + w * ac[k];
  } else if (va <= 0 && (d4 - d3) >= 0 && (d5 - d6) >= 0) {
    const T w = (d4 - d3) / ((d4 - d3) + (d5 - d6));
    for (int k = 0; k < 3; k++) q[k] = b[k] + w * (c[k] - b[k]);
  } else {
    const T denom = T(1) / (va + vb + vc);
    const T v = vb * denom, w = vc * denom;
    for (int k = 0; k < 3; k++) q[k] = a[k] + ab[k] * v + ac[k] * w;
  }
  for (int k = 0; k < 3; k++) qf[k] = (float)q[k];
  return (float)dot(q, q);
}
__device__ __forceinline__ void find_pos(const MPoint& P0, const MPoint& P1, const MPoint& P2, const MPoint& P3,
                                         float* pos) {
  float dir[3];
  portal_dir(P1, P2, P3, dir);
  float b0, b1, b2, b3, t[3];
  cross3(t, P2.v, P3.v); b0 = dot3(P1.v, t);
  cross3(t, P2.v, P0.v); b1 = dot3(P3.v, t);
  cross3(t, P1.v, P3.v); b2 = dot3(P0.v, t);
  cross3(t, P1.v, P0.v); b3 = dot3(P2.v, t);
  float sum = b0 + b1 + b2 + b3;
  if (sum <= 0) {
    b0 = 0;
    cross3(t, P3.v, dir); b1 = dot3(P2.v, t);
    cross3(t, P1.v, dir); b2 = dot3(P3.v, t);
    cross3(t, P2.v, dir); b3 = dot3(P1.v, t);
    sum = b1 + b2 + b3;
  }
  float inv = 1.0f / sum;
  for (int k = 0; k < 3; k++) {
    float p1 = b0 * P0.a[k] + b1 * P1.a[k] + b2 * P2.a[k] + b3 * P3.a[k];
    float p2 = b0 * P0.b[k] + b1 * P1.b[k] + b2 * P2.b[k] + b3 * P3.b[k];
    pos[k] = 0.5f * (p1 + p2) * inv;
  }
}

// Shape of geom g from its record (two memory round trips: record, then body pose in LDS).
template <class Ctx>
__device__ __forceinline__ void make_shape_rec(const Ctx& c, int g, float half_margin, Shape& s) {
  const DevModel& m = c.mdl();
  const DXG float4* r = m.geom_rec + 8 * g;
  float4 r0 = r[0], r1 = r[1], r2 = r[2], r3 = r[3], r4 = r[4], r5 = r[5], r6 = r[6];
  s.type = __float_as_int(r0.x);
  int b = __float_as_int(r0.y);
  s.nvert = __float_as_int(r0.z);
  s.bin_n = __float_as_int(r0.w);
  s.bin_cap = __float_as_int(r1.x);
  s.vert4 = m.mesh_vert4 + __float_as_int(r1.y);
  s.bin4 = m.mesh_bin4 + __float_as_int(r1.z);
  s.size[0] = r2.x; s.size[1] = r2.y; s.size[2] = r2.z;
  const float gpos[3] = {r3.x, r3.y, r3.z};
  const float gmat[9] = {r4.x, r4.y, r4.z, r4.w, r5.x, r5.y, r5.z, r5.w, r6.x};
  const float gc[3] = {r6.y, r6.z, r6.w};
  const float* xp = c.f(c.L.xpos) + 3 * b;
  const float* xm = c.f(c.L.xmat) + 9 * b;
  float t[3];
  matvec3(t, xm, gpos);
  s.pos[0] = xp[0] + t[0]; s.pos[1] = xp[1] + t[1]; s.pos[2] = xp[2] + t[2];
  matmul3(s.mat, xm, gmat);
  matvec3(t, s.mat, gc);
  s.center[0] = s.pos[0] + t[0]; s.center[1] = s.pos[1] + t[1]; s.center[2] = s.pos[2] + t[2];
  s.margin = half_margin;
}

// Narrowphase runs DX_WAVE / NPG candidate pairs per wave, one per NPG-lane group (part of a DPP
// row).  Every lane of a group runs the same MPR control flow for its pair; the
// groups diverge only through the exec mask.
// NPG lanes per group: 8 (two groups per DPP row) or 4 (see narrow_pass).
// The group size is a template parameter (NPG = 8: eight pairs per wave; NPG = 4:
// sixteen, for substeps with more than eight candidates, see collision()).
template <int NPG> __device__ __forceinline__ int sl_() { return LANE & (NPG - 1); }
template <int NPG> __device__ __forceinline__ int gbase_() { return LANE & (DX_WAVE - NPG); }  // first lane of the group
#define SL sl_<NPG>()
#define GBASE gbase_<NPG>()
template <int NPG>
__device__ __forceinline__ int row_max_i(int m) {
  m = max(m, dpp_i<0xB1, 0xF>(m));                      // quad_perm [1,0,3,2]
  if (NPG >= 4) m = max(m, dpp_i<0x4E, 0xF>(m));        // quad_perm [2,3,0,1]
  if (NPG >= 8) m = max(m, dpp_i<0x141, 0xF>(m));       // row_half_mirror (8 lanes)
  if (NPG == 16) m = max(m, dpp_i<0x140, 0xF>(m));      // row_mirror (16 lanes)
  return m;
}
template <int NPG>
__device__ __forceinline__ int row_or_i(int m) {
  m |= dpp_i<0xB1, 0xF>(m);
  if (NPG >= 4) m |= dpp_i<0x4E, 0xF>(m);
  if (NPG >= 8) m |= dpp_i<0x141, 0xF>(m);
  if (NPG == 16) m |= dpp_i<0x140, 0xF>(m);
  return m;
}
template <int NPG>
__device__ __forceinline__ int row_min_i(int m) {
  m = min(m, dpp_i<0xB1, 0xF>(m));
  if (NPG >= 4) m = min(m, dpp_i<0x4E, 0xF>(m));
  if (NPG >= 8) m = min(m, dpp_i<0x141, 0xF>(m));
  if (NPG == 16) m = min(m, dpp_i<0x140, 0xF>(m));
  return m;
}

// Local-frame support of a primitive (box, sphere, capsule) in local direction ld.
__device__ __forceinline__ void support_prim(const Shape& s, const float* ld, float* lp) {
  lp[0] = lp[1] = lp[2] = 0;
  if (s.type == DXG_BOX) {
    for (int k = 0; k < 3; k++) lp[k] = ld[k] >= 0 ? s.size[k] : -s.size[k];
  } else if (s.type == DXG_SPHERE || s.type == DXG_CAPSULE) {
    float n = norm3(ld);
    if (n > 1e-20f) { float sc = s.size[0] / n; lp[0] = ld[0] * sc; lp[1] = ld[1] * sc; lp[2] = ld[2] * sc; }
    if (s.type == DXG_CAPSULE) lp[2] += ld[2] >= 0 ? s.size[1] : -s.size[1];
  }
}
// local support -> world point, plus the shape's half margin along dir
__device__ __forceinline__ void support_world(const Shape& s, const float* lp, const float* dir, float* out) {
  matvec3(out, s.mat, lp);
  out[0] += s.pos[0]; out[1] += s.pos[1]; out[2] += s.pos[2];
  if (s.margin > 0) {
    float n = norm3(dir);
    if (n > 1e-20f) {
      float sc = s.margin / n;
      out[0] += dir[0] * sc; out[1] += dir[1] * sc; out[2] += dir[2] * sc;
    }
  }
}
// Hull scan state of one lane: its first maximal slot (strict '>') and coordinates.
struct HullBest {
  float d, x, y, z;
  int i;
};
__device__ __forceinline__ void hull_take(HullBest& h, float4 v, float d, int i, bool ok) {
  bool t = ok && d > h.d;
  h.d = t ? d : h.d;
  h.i = t ? i : h.i;
  h.x = t ? v.x : h.x;
  h.y = t ? v.y : h.y;
  h.z = t ? v.z : h.z;
}
// Group reduction: the lowest vertex index among the lanes holding the maximum (a
// cell's list is sorted by vertex index, a whole hull is scanned in index order, so
// this is the vertex the oracle's serial scan returns); its coordinates reach the group
// by a DPP or over the group in which every other lane offers 0 (one lane holds the
// winning slot: the indices of a group's slots are distinct) -- no ballot and no
// ds_bpermute round trip.  The maximum runs on order-preserving integers (f2ord), every
// step one v_*_dpp instruction.
template <int NPG>
__device__ __forceinline__ void hull_reduce(const HullBest& h, float* lp) {
  const int kd = f2ord(h.d);
  const int kmax = row_max_i<NPG>(kd);
  const int bi = row_min_i<NPG>(kd == kmax ? h.i : 0x7fffffff);
  const bool win = kd == kmax && h.i == bi;
  lp[0] = __int_as_float(row_or_i<NPG>(win ? __float_as_int(h.x) : 0));
  lp[1] = __int_as_float(row_or_i<NPG>(win ? __float_as_int(h.y) : 0));
  lp[2] = __int_as_float(row_or_i<NPG>(win ? __float_as_int(h.z) : 0));
}
// Cube-map cell of local direction ld (host twin: dx_api.hip cell_corners).  Returns
// -1 for a zero direction (then the whole hull is scanned, as the oracle does).  No
// branch: every lane computes a cell and selects -1 after.
__device__ __forceinline__ int hull_cell(const float* ld, int n) {
  float ax0 = fabsf(ld[0]), ax1 = fabsf(ld[1]), ax2 = fabsf(ld[2]);
  int ax = (ax0 >= ax1 && ax0 >= ax2) ? 0 : (ax1 >= ax2 ? 1 : 2);
  float a = ax == 0 ? ld[0] : (ax == 1 ? ld[1] : ld[2]);
  float u = ax == 0 ? ld[1] : (ax == 1 ? ld[2] : ld[0]);
  float v = ax == 0 ? ld[2] : (ax == 1 ? ld[0] : ld[1]);
  const float aa = fabsf(a);
  const bool nz = aa > 1e-30f;
  const float inv = 1.0f / (nz ? aa : 1.f);
  int iu = (int)((u * inv + 1.0f) * 0.5f * (float)n);
  int iv = (int)((v * inv + 1.0f) * 0.5f * (float)n);
  iu = min(max(iu, 0), n - 1);
  iv = min(max(iv, 0), n - 1);
  int face = 2 * ax + (a < 0 ? 1 : 0);
  return nz ? (face * n + iu) * n + iv : -1;
}
// One hull's support scan by a lane group.  First a DX_HULL_K-slot block -- the
// direction's cube-map cell (dx_api.hip build_hull_bins), or the first K vertices of a
// hull that is not binned / a zero direction -- one 128-B line, one memory round trip;
// then, rarely, an overflow run: the rest of a cell whose slot K - 1 is a header, or the
// rest of a whole-hull scan.
struct HullScan {
  HullBest h;
  const DXG float4* ov;  // overflow run (a valid address even when empty)
  int nov;               // its slots
  bool cell;             // cell scan: the vertex index is the slot's w; else the slot number
};
__device__ __forceinline__ void hull_block(const Shape& s, const float* ld, const DXG float4*& blk, int& n1, bool& cell) {
  const int c = s.bin_n > 0 ? hull_cell(ld, max(s.bin_n, 1)) : -1;  // (selects, no branch)
  cell = c >= 0;
  blk = cell ? s.bin4 + DX_HULL_K * c : s.vert4;
  n1 = cell ? DX_HULL_K : min(s.nvert, DX_HULL_K);
}
template <int NPG>
__device__ __forceinline__ void hull_take_block(const Shape& s, const float* ld, const float4 (&v)[DX_HULL_K / NPG],
                                                const DXG float4* blk, int n1, bool cell, HullScan& H) {
  constexpr int DX_SLK = DX_HULL_K / NPG;  // block slots per lane
#pragma unroll
  for (int u = 0; u < DX_SLK; u++) {
    const int sl = u * NPG + SL;
    const int idx = __float_as_int(v[u].w);  // (cells and whole-hull slots alike)
    hull_take(H.h, v[u], v[u].x * ld[0] + v[u].y * ld[1] + v[u].z * ld[2], idx, sl < n1 && idx >= 0);
  }
  // slot K - 1 (the group's last lane, last load) of a cell: a header (index -2) names
  // the overflow run.  The header is rare: the lanes that hold one are found by ballot
  // and only then is it broadcast to its group.
  H.cell = cell;
  H.ov = blk;
  H.nov = 0;
  const bool hdr = cell && SL == NPG - 1 && __float_as_int(v[DX_SLK - 1].w) == -2;
  if (__any(hdr)) {
    const int src = GBASE | (NPG - 1);
    const int tag = __shfl(__float_as_int(v[DX_SLK - 1].w), src, 64);
    const int off = __shfl(__float_as_int(v[DX_SLK - 1].x), src, 64);
    const int cnt = __shfl(__float_as_int(v[DX_SLK - 1].y), src, 64);
    if (cell && tag == -2) {
      H.ov = s.bin4 + off;
      H.nov = cnt - (DX_HULL_K - 1);
    }
  }
  if (!cell && s.nvert > DX_HULL_K) {
    H.ov = s.vert4 + DX_HULL_K;
    H.nov = s.nvert - DX_HULL_K;
  }
}
template <int NPG>
__device__ __forceinline__ void hull_take_run(const float* ld, const float4 (&v)[DX_HULL_K / NPG], int base, HullScan& H) {
#pragma unroll
  for (int u = 0; u < DX_HULL_K / NPG; u++) {
    const int sl = base + u * NPG + SL;
    const int idx = __float_as_int(v[u].w);  // (cells and whole-hull slots alike)
    hull_take(H.h, v[u], v[u].x * ld[0] + v[u].y * ld[1] + v[u].z * ld[2], idx, sl < H.nov && idx >= 0);
  }
}

// Support points of A along dir and of B along -dir, by one lane group split in halves:
// lanes 0-3 of a group hold A (the pair's first geom) in their Shape and scan its hull
// block along dir, lanes 4-7 hold B and scan along -dir, two slots each; the halves swap
// their world points at the end (DPP row_half_mirror: lane i <-> 7 - i).  Every lane
// computes one cube-map cell, one local direction, one reduction (over its quad: two DPP
// steps) and one world transform, and keeps one Shape.  The vertex arithmetic and the
// first-maximiser rule are those of the oracle's serial scan.
// (NPG = 4: two lanes per half, four slots each, halves swapped by quad_perm [2,3,0,1])
template <int NPG> __device__ __forceinline__ bool half_b() { return (SL & (NPG / 2)) != 0; }  // this lane holds B
// the other half's value: lane i <-> 7 - i (NPG 8) or i ^ 2 (NPG 4)
template <int NPG> __device__ __forceinline__ float half_swap(float v) {
  static_assert(NPG == 8 || NPG == 4, "groups of 8 or 4 lanes");
  return NPG == 8 ? dpp_f<0x141, 0xF>(v) : dpp_f<0x4E, 0xF>(v);
}
// the narrowphase trip's clock (DX_NP_MARKS builds): stage_mark from divergent code, the first active lane keeping the time
struct NpClock {
  unsigned long long* acc;
  int* I;
  __device__ void mark(int k) const {
    if (DX_NP_MARKS && acc && LANE == __builtin_amdgcn_readfirstlane(LANE)) {
      unsigned long long t = __builtin_amdgcn_s_memtime();
      unsigned long long* last = (unsigned long long*)(I + 10);
      stage_add(acc + k, t - *last);
      *last = t;
    }
  }
};
template <int NPG>
__device__ __forceinline__ void support_pair(const Shape& S, const float* dir, float* outA, float* outB,
                                             const NpClock& ck = NpClock{nullptr, nullptr}) {
  constexpr int H = NPG / 2;          // lanes per half
  constexpr int DX_SLH = DX_HULL_K / H;  // block slots per lane of a half group
  const bool hb = half_b<NPG>();
  const int q = SL & (H - 1);
  const float sg = hb ? -1.f : 1.f;
  const float d[3] = {sg * dir[0], sg * dir[1], sg * dir[2]};
  float ld[3];
  mattvec3(ld, S.mat, d);
  const int type = S.type;
  float lp[3];
  if (__any(type == DXG_MESH)) {
    const Shape& s = S;
    const bool mesh = type == DXG_MESH;
    HullBest h = {-3.0e38f, 0.f, 0.f, 0.f, 0x7fffffff};
    const DXG float4* blk;
    int n1;
    bool cell;
    hull_block(s, ld, blk, n1, cell);  // (every lane: a primitive's record has no cells)
    n1 = mesh ? n1 : 0;
    cell = mesh && cell;
    float4 v[DX_SLH];
#pragma unroll
    for (int u = 0; u < DX_SLH; u++) {
      const int sl = H * u + q;
      v[u] = blk[sl < n1 ? sl : 0];
    }
    // the lane's first maximiser among its slots (a lane's slots are in vertex-index
    // order): every dot at once, a max tree, then the selects from the last slot down --
    // not a chain of DX_SLH dependent compare-and-keep steps
    {
      float dd[DX_SLH];
      int ix[DX_SLH];
#pragma unroll
      for (int u = 0; u < DX_SLH; u++) {
        const int sl = H * u + q;
        const int idx = __float_as_int(v[u].w);  // (cells and whole-hull slots alike)
        const bool ok = mesh && sl < n1 && idx >= 0;
        dd[u] = ok ? v[u].x * ld[0] + v[u].y * ld[1] + v[u].z * ld[2] : -3.0e38f;
        ix[u] = ok ? idx : 0x7fffffff;
      }
      float m = dd[0];
#pragma unroll
      for (int u = 1; u < DX_SLH; u++) m = fmaxf(m, dd[u]);
      h.d = m;
      h.i = ix[DX_SLH - 1];
      h.x = v[DX_SLH - 1].x;
      h.y = v[DX_SLH - 1].y;
      h.z = v[DX_SLH - 1].z;
#pragma unroll
      for (int u = DX_SLH - 2; u >= 0; u--) {
        const bool t = dd[u] == m;
        h.i = t ? ix[u] : h.i;
        h.x = t ? v[u].x : h.x;
        h.y = t ? v[u].y : h.y;
        h.z = t ? v[u].z : h.z;
      }
    }
    ck.mark(ST_NP_SUPLOAD);
    // overflow run: slot K - 1 of a cell (its half's last lane, last load) may be a header
    const DXG float4* ov = blk;
    int nov = 0;
    const bool hdr = mesh && cell && q == H - 1 && __float_as_int(v[DX_SLH - 1].w) == -2;
    if (__any(hdr)) {
      const int src = (LANE & ~(H - 1)) | (H - 1);
      const int tag = __shfl(__float_as_int(v[DX_SLH - 1].w), src, 64);
      const int off = __shfl(__float_as_int(v[DX_SLH - 1].x), src, 64);
      const int cnt = __shfl(__float_as_int(v[DX_SLH - 1].y), src, 64);
      if (mesh && cell && tag == -2) {
        ov = s.bin4 + off;
        nov = cnt - (DX_HULL_K - 1);
      }
    }
    if (mesh && !cell && s.nvert > DX_HULL_K) {
      ov = s.vert4 + DX_HULL_K;
      nov = s.nvert - DX_HULL_K;
    }
    for (int base = 0; __any(base < nov); base += DX_HULL_K) {
#pragma unroll
      for (int u = 0; u < DX_SLH; u++) {
        const int sl = base + H * u + q;
        v[u] = ov[sl < nov ? sl : 0];
      }
#pragma unroll
      for (int u = 0; u < DX_SLH; u++) {
        const int sl = base + H * u + q;
        const int idx = __float_as_int(v[u].w);  // (cells and whole-hull slots alike)
        hull_take(h, v[u], v[u].x * ld[0] + v[u].y * ld[1] + v[u].z * ld[2], idx, sl < nov && idx >= 0);
      }
    }
    // half reduction: the lowest vertex index among the maxima, its coordinates by a DPP
    // or in which only the winning lane offers its own (hull_reduce)
    const int kd = f2ord(h.d);
    int kmax = max(kd, dpp_i<0xB1, 0xF>(kd));
    if (H == 4) kmax = max(kmax, dpp_i<0x4E, 0xF>(kmax));
    int bi = kd == kmax ? h.i : 0x7fffffff;
    bi = min(bi, dpp_i<0xB1, 0xF>(bi));
    if (H == 4) bi = min(bi, dpp_i<0x4E, 0xF>(bi));
    const bool win = kd == kmax && h.i == bi;
    int hx = win ? __float_as_int(h.x) : 0, hy = win ? __float_as_int(h.y) : 0, hz = win ? __float_as_int(h.z) : 0;
    hx |= dpp_i<0xB1, 0xF>(hx);
    hy |= dpp_i<0xB1, 0xF>(hy);
    hz |= dpp_i<0xB1, 0xF>(hz);
    if (H == 4) {
      hx |= dpp_i<0x4E, 0xF>(hx);
      hy |= dpp_i<0x4E, 0xF>(hy);
      hz |= dpp_i<0x4E, 0xF>(hz);
    }
    if (mesh) { lp[0] = __int_as_float(hx); lp[1] = __int_as_float(hy); lp[2] = __int_as_float(hz); }
  }
  if (type != DXG_MESH) support_prim(S, ld, lp);
  // world point (+ the half margin along this half's direction), then the halves swap
  float out[3];
  support_world(S, lp, d, out);
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const float o = half_swap<NPG>(out[k]);  // the other half's point
    outA[k] = hb ? o : out[k];
    outB[k] = hb ? out[k] : o;
  }
}

// Support of one shape along dir (group-cooperative for hulls).
template <int NPG>
__device__ __forceinline__ void support_grp(const Shape& s, const float* dir, float* out) {
  constexpr int DX_SLK = DX_HULL_K / NPG;
  float ld[3], lp[3];
  mattvec3(ld, s.mat, dir);
  if (s.type == DXG_MESH) {
    const DXG float4* blk;
    int n1;
    bool cell;
    hull_block(s, ld, blk, n1, cell);
    HullScan S;
    S.h = {-3.0e38f, 0.f, 0.f, 0.f, 0x7fffffff};
    float4 v[DX_SLK];
#pragma unroll
    for (int u = 0; u < DX_SLK; u++) {
      const int sl = u * NPG + SL;
      v[u] = blk[sl < n1 ? sl : 0];
    }
    hull_take_block<NPG>(s, ld, v, blk, n1, cell, S);
    for (int base = 0; __any(base < S.nov); base += DX_HULL_K) {
#pragma unroll
      for (int u = 0; u < DX_SLK; u++) {
        const int sl = base + u * NPG + SL;
        v[u] = S.ov[sl < S.nov ? sl : 0];
      }
      if (base < S.nov) hull_take_run<NPG>(ld, v, base, S);
    }
    hull_reduce<NPG>(S.h, lp);
  } else {
    support_prim(s, ld, lp);
  }
  support_world(s, lp, dir, out);
}

struct NpStats { int support, mpr, hit, plane_box, plane_convex, capsule, maxit; };

// MPR penetration on A - B (libccd ccdMPRPenetration structure, see the oracle's
// mpr_penetration) as a resumable state machine: one support evaluation per
// mpr_step, so the lane groups of a wave -- each on its own pair and in its
// own MPR phase -- share every support pass.  The portal points live in LDS (36
// words per group: P0..P3 = v, a, b): kept in registers, every divergent phase
// branch re-materialised all 36 of them at its join.
//   phase 0: P1          phase 1: P2          phase 2: portal discovery (P3)
//   phase 3: portal refinement towards the origin
//   phase 4: refinement of the penetration (contact) portal
#define MP_WORDS 36
__device__ __forceinline__ void mp_st(float* d, const MPoint& p) {
#pragma unroll
  for (int k = 0; k < 3; k++) { d[k] = p.v[k]; d[3 + k] = p.a[k]; d[6 + k] = p.b[k]; }
}
__device__ __forceinline__ void mp_ld(const float* d, MPoint& p) {
#pragma unroll
  for (int k = 0; k < 3; k++) { p.v[k] = d[k]; p.a[k] = d[3 + k]; p.b[k] = d[6 + k]; }
}
__device__ __forceinline__ void v3sel(float* d, const float* s, bool c) {
  d[0] = c ? s[0] : d[0]; d[1] = c ? s[1] : d[1]; d[2] = c ? s[2] : d[2];
}
__device__ __forceinline__ void portal_dir_v(const float* v1, const float* v2, const float* v3, float* dir) {
  float a[3], b[3];
  sub3(a, v2, v1);
  sub3(b, v3, v1);
  cross3(dir, a, b);
  normalize3(dir);
}
struct MprState {
  float* P;  // this group's 36 LDS words
  float dir[3];
  int phase, it;
};
// cached: a separating direction of this pair from an earlier collision pass (world
// frame), tried first (phase -1).  The cache may only save work, never change a result:
// its entries are stored plainly and shared by two pairs per slot, so which entry a task
// sees depends on the narrowphase layout and on which XCD ran the env's last substep.
// The cached test therefore returns "separated" only when the Minkowski difference lies
// at least DX_SEP_CLEAR beyond the origin along the cached direction: every point MPR
// can put into a portal is a point of A - B, so MPR's own verdict is then "separated"
// too, unless fp32 rounding in its portal tests exceeded DX_SEP_CLEAR (coordinates
// ~0.3 m: ~1e-7).  Anything closer falls through to MPR from its standard start, with
// the very direction an uncached pair starts from (kept in the P1 slot, unused until
// phase 0 writes it) -- so the pair's arithmetic is then exactly the uncached one.
#define DX_SEP_CLEAR 1e-5f
template <int NPG>
__device__ __forceinline__ void mpr_init(const Shape& G, MprState& S, const float* cached) {
  MPoint P0;
  const bool hb = half_b<NPG>();
  for (int k = 0; k < 3; k++) {
    const float o = half_swap<NPG>(G.center[k]);  // the other half's shape centre
    P0.a[k] = hb ? o : G.center[k];
    P0.b[k] = hb ? G.center[k] : o;
  }
  sub3(P0.v, P0.a, P0.b);
  if (fzero(P0.v[0]) && fzero(P0.v[1]) && fzero(P0.v[2])) P0.v[0] += 1e-9f;
  mp_st(S.P, P0);
  S.dir[0] = -P0.v[0]; S.dir[1] = -P0.v[1]; S.dir[2] = -P0.v[2];
  normalize3(S.dir);
  S.phase = 0;
  S.it = 0;
  if (cached) {
    S.P[9] = S.dir[0]; S.P[10] = S.dir[1]; S.P[11] = S.dir[2];  // the uncached start
    S.dir[0] = cached[0]; S.dir[1] = cached[1]; S.dir[2] = cached[2];
    S.phase = -1;
  }
}
// Returns 0: running, 1: separated (no contact), 2: penetration (depth/normal/pos set).
// The eight groups of a wave are in different MPR phases on most trips, so the phases
// share one code path: every phase's next direction is normalize(cross(A - C, B - C))
// (or -v0) with its operands selected per group, and the new support point goes to one
// portal slot chosen per group.  Each phase performs exactly the arithmetic of libccd's
// structure (the oracle's dxo_mpr), so the results are unchanged; only the separated,
// degenerate and final exits branch.
template <int NPG>
__device__ __forceinline__ int mpr_step(const Shape& G, MprState& S, float& depth, float* normal,
                                        float* pos, NpStats& st, const NpClock& ck = NpClock{nullptr, nullptr}) {
  const float tol = 1e-6f;
  const int maxit = 50;
  float* P = S.P;
  float v0[3], v1[3], v2[3], v3[3];  // portal vertices (read before the support's memory round trip)
  for (int k = 0; k < 3; k++) { v0[k] = P[k]; v1[k] = P[9 + k]; v2[k] = P[18 + k]; v3[k] = P[27 + k]; }
  MPoint p;
  float* dir = S.dir;
  support_pair<NPG>(G, dir, p.a, p.b, ck);
  ck.mark(ST_NP_SUPRED);
  sub3(p.v, p.a, p.b);
  st.support++;
  const int ph = S.phase;
  const float dt = dot3(p.v, dir);  // (phases 3 and 4: dv4)
  const bool behind = fzero(dt) || dt < 0;
  if (ph >= 3 && S.it > maxit) st.maxit++;
  const bool stop =
      fminf(dt - dot3(v1, dir), fminf(dt - dot3(v2, dir), dt - dot3(v3, dir))) <= tol || S.it > maxit;
  // exits: separated (phases -1..3) and converged penetration (phase 4)
  if ((ph == -1 && dt < -DX_SEP_CLEAR) || (ph >= 0 && ph <= 1 && behind) || (ph == 2 && (S.it > 1000 || behind)) ||
      (ph == 3 && (stop || dt < 0)))
    return 1;
  if (ph == 4 && stop) {
    float cl[3];
    float d2 = tri_origin_dist2_t<double>(v1, v2, v3, cl);
    depth = sqrtf(d2);
    if (depth > 1e-20f) {
      float sc = 1.0f / depth;
      normal[0] = cl[0] * sc; normal[1] = cl[1] * sc; normal[2] = cl[2] * sc;
    } else {
      normal[0] = dir[0]; normal[1] = dir[1]; normal[2] = dir[2];
    }
    MPoint Q0, Q1, Q2, Q3;
    mp_ld(P, Q0); mp_ld(P + 9, Q1); mp_ld(P + 18, Q2); mp_ld(P + 27, Q3);
    find_pos(Q0, Q1, Q2, Q3, pos);
    return 2;
  }
  // phase 2 (portal discovery): does p replace P2 (r2) or P1 (r1)?
  float t[3];
  cross3(t, v1, p.v);
  float dd = dot3(t, v0);
  const bool r2 = ph == 2 && dd < 0 && !fzero(dd);
  cross3(t, p.v, v2);
  dd = dot3(t, v0);
  const bool r1 = ph == 2 && !r2 && dd < 0 && !fzero(dd);
  // phases 3 / 4 (expand_portal): which vertex p replaces
  float v4v0[3];
  cross3(v4v0, p.v, v0);
  const bool c1 = dot3(v1, v4v0) > 0, c2 = dot3(v2, v4v0) > 0, c3 = dot3(v3, v4v0) > 0;
  const bool x1 = ph >= 3 && (c1 ? c2 : !c3), x2 = ph >= 3 && !c1 && c3, x3 = ph >= 3 && c1 && !c2;
  // portal vertices after this step (registers; the LDS slots are written below)
  v3sel(v1, p.v, r1 || x1);
  v3sel(v2, p.v, r2 || x2);
  v3sel(v3, p.v, x3);
  // next direction: X = cross(a - c, b - c)
  //   0: (v0, p, 0)   1: (v1, p, v0)   2: (v1', v2', v0) if p replaced P1/P2, else (v2, p, v1)
  //   3/4: (v2', v3', v1')   -1: X = -v0
  const bool rr = r1 || r2;
  float a[3], b[3], cc[3];
  for (int k = 0; k < 3; k++) {
    a[k] = ph == 0 ? v0[k] : (ph == 1 || (ph == 2 && rr)) ? v1[k] : v2[k];
    b[k] = ph >= 3 ? v3[k] : (ph == 2 && rr) ? v2[k] : p.v[k];
    cc[k] = ph == 0 ? 0.f : (ph == 1 || ph == 2 && rr) ? v0[k] : v1[k];
  }
  float ea[3], eb[3];
  sub3(ea, a, cc);
  sub3(eb, b, cc);
  float X[3];
  cross3(X, ea, eb);
  if (ph == 0 && fzero(dot3(X, X))) {  // p on the line through the origin and v0
    dir[0] = X[0]; dir[1] = X[1]; dir[2] = X[2];
    if (fzero(p.v[0]) && fzero(p.v[1]) && fzero(p.v[2])) {
      depth = 0;
      normal[0] = 0; normal[1] = 0; normal[2] = 1;
    } else {
      depth = norm3(p.v);
      for (int k = 0; k < 3; k++) normal[k] = p.v[k];
      normalize3(normal);
    }
    for (int k = 0; k < 3; k++) pos[k] = 0.5f * (p.a[k] + p.b[k]);
    return 2;
  }
  normalize3(X);
  if (ph == -1) { X[0] = v1[0]; X[1] = v1[1]; X[2] = v1[2]; }  // not clear: MPR's own start (mpr_init)
  // phase 1: orient the portal so that the origin is on dir's side (swap P1, P2)
  const bool swap = ph == 1 && dot3(X, v0) > 0;
  if (swap) {
    MPoint q;
    mp_ld(P + 9, q);
    mp_st(P + 18, q);
    X[0] = -X[0]; X[1] = -X[1]; X[2] = -X[2];
  }
  dir[0] = X[0]; dir[1] = X[1]; dir[2] = X[2];
  // the new support point's slot: 0 -> P1; 1 -> P2 (P1 on a swap); 2 -> P3 (and P1 or
  // P2 when it replaces one); 3 / 4 -> the replaced vertex
  const int slot = (ph == 0 || swap || x1) ? 1 : (ph == 1 || x2) ? 2 : 3;
  if (ph >= 0) mp_st(P + 9 * slot, p);
  if (rr) mp_st(P + (r2 ? 18 : 9), p);
  // phase bookkeeping
  if (ph == -1) {
    S.phase = 0;
  } else if (ph == 0) {
    S.phase = 1;
  } else if (ph == 1) {
    S.phase = 2;
    S.it = 0;
  } else if (ph == 2) {
    S.it++;
    if (!rr) {
      S.phase = dot3(dir, v1) >= 0 ? 4 : 3;
      S.it = 0;
    }
  } else {
    S.it++;
    if (ph == 3 && dot3(dir, v1) >= 0) { S.phase = 4; S.it = 0; }
  }
  return 0;
}

__device__ __forceinline__ bool sphere_overlap(const float* c1, float r1, const float* c2, float r2, float margin) {
  float t[3];
  sub3(t, c1, c2);
  float rr = r1 + r2 + margin;
  return dot3(t, t) <= rr * rr;
}

// Separating-axis test of two oriented boxes (Gottschalk's 15 axes), inflated by margin.
// obb: [centre(3) in body frame, R(9) body<-box, half extents(3)].
__device__ __forceinline__ bool obb_overlap(const float* o1, const float* xp1, const float* xm1, const float* o2,
                            const float* xp2, const float* xm2, float margin) {
  float ca[3], cb[3], Ra[9], Rb[9];
  matvec3(ca, xm1, o1);
  matvec3(cb, xm2, o2);
  for (int k = 0; k < 3; k++) { ca[k] += xp1[k]; cb[k] += xp2[k]; }
  matmul3(Ra, xm1, o1 + 3);
  matmul3(Rb, xm2, o2 + 3);
  const float* ea = o1 + 12;
  const float* eb = o2 + 12;
  float t0[3] = {cb[0] - ca[0], cb[1] - ca[1], cb[2] - ca[2]};
  float t[3], R[9], AR[9];
  // t in a's frame, R = Ra^T Rb
  for (int i = 0; i < 3; i++) {
    t[i] = Ra[i] * t0[0] + Ra[3 + i] * t0[1] + Ra[6 + i] * t0[2];
    for (int j = 0; j < 3; j++) {
      R[3 * i + j] = Ra[i] * Rb[j] + Ra[3 + i] * Rb[3 + j] + Ra[6 + i] * Rb[6 + j];
      AR[3 * i + j] = fabsf(R[3 * i + j]) + 1e-6f;
    }
  }
  for (int i = 0; i < 3; i++) {
    float rb = eb[0] * AR[3 * i] + eb[1] * AR[3 * i + 1] + eb[2] * AR[3 * i + 2];
    if (fabsf(t[i]) > ea[i] + rb + margin) return false;
  }
  for (int j = 0; j < 3; j++) {
    float ra = ea[0] * AR[j] + ea[1] * AR[3 + j] + ea[2] * AR[6 + j];
    float tj = t[0] * R[j] + t[1] * R[3 + j] + t[2] * R[6 + j];
    if (fabsf(tj) > ra + eb[j] + margin) return false;
  }
  for (int i = 0; i < 3; i++) {
    int i1 = (i + 1) % 3, i2 = (i + 2) % 3;
    for (int j = 0; j < 3; j++) {
      int j1 = (j + 1) % 3, j2 = (j + 2) % 3;
      float ra = ea[i1] * AR[3 * i2 + j] + ea[i2] * AR[3 * i1 + j];
      float rb = eb[j1] * AR[3 * i + j2] + eb[j2] * AR[3 * i + j1];
      float tt = t[i2] * R[3 * i1 + j] - t[i1] * R[3 * i2 + j];
      if (fabsf(tt) > ra + rb + margin) return false;
    }
  }
  return true;
}

// Overlap of two boxes given in their bodies' frames (axes = body axes): centre c,
// half extents e, body pose (xp, xm); the 15-axis SAT of obb_overlap.
__device__ __forceinline__ bool box_overlap(const float* c1, const float* e1, const float* xp1, const float* xm1,
                                            const float* c2, const float* e2, const float* xp2, const float* xm2,
                                            float margin) {
  const float o1[15] = {c1[0], c1[1], c1[2], 1.f, 0.f, 0.f, 0.f, 1.f, 0.f, 0.f, 0.f, 1.f, e1[0], e1[1], e1[2]};
  const float o2[15] = {c2[0], c2[1], c2[2], 1.f, 0.f, 0.f, 0.f, 1.f, 0.f, 0.f, 0.f, 1.f, e2[0], e2[1], e2[2]};
  return obb_overlap(o1, xp1, xm1, o2, xp2, xm2, margin);
}

// Appends one contact record (called by a single lane).
__device__ __forceinline__ void write_contact(float* con, int slot, const float* pos, const float* n, float dist, int gp) {
  float* r = con + DX_CON_STRIDE * slot;
  r[0] = pos[0]; r[1] = pos[1]; r[2] = pos[2];
  // frame: normal, tangent ([3P] mju_makeFrame)
  float y[3];
  if (fabsf(n[1]) < 0.5f) { y[0] = 0; y[1] = 1; y[2] = 0; }
  else { y[0] = 0; y[1] = 0; y[2] = 1; }
  float t = n[0] * y[0] + n[1] * y[1] + n[2] * y[2];
  y[0] -= t * n[0]; y[1] -= t * n[1]; y[2] -= t * n[2];
  normalize3(y);
  float z[3];
  cross3(z, n, y);
  r[3] = n[0]; r[4] = n[1]; r[5] = n[2];
  r[6] = y[0]; r[7] = y[1]; r[8] = y[2];
  r[9] = z[0]; r[10] = z[1]; r[11] = z[2];
  r[12] = dist;
  r[13] = __int_as_float(gp);
}

// One lane's share of a group's narrowphase result: `wr` lanes write a contact at
// (group offset + rank).
struct NpOut {
  bool wr;
  int rank;
  float pos[3], n[3], dist;
};

// True for pairs the primitive routines handle (plane-*, capsule-capsule); the rest
// (box/mesh/sphere/capsule vs box/mesh) go through MPR.
__device__ __forceinline__ bool pair_is_prim(const DevModel& m, int gp) {
  int t1 = m.geom_type[m.gpair_geom[2 * gp]], t2 = m.geom_type[m.gpair_geom[2 * gp + 1]];
  return t1 == DXG_PLANE || (t1 == DXG_CAPSULE && t2 == DXG_CAPSULE);
}
// Primitive narrowphase of one geom pair by one lane group; returns the group's
// contact count (group-uniform, at most 4).
template <int NPG, class Ctx>
__device__ __forceinline__ int narrowphase_prim(const Ctx& c, int gp, NpOut& o, NpStats& st) {
  const DevModel& m = c.mdl();
  int g1 = m.gpair_geom[2 * gp], g2 = m.gpair_geom[2 * gp + 1];
  int t1 = m.geom_type[g1], t2 = m.geom_type[g2];
  float margin = m.gpair_margin[gp];
  o.wr = false;
  o.rank = 0;
  if (t1 == DXG_PLANE) {
    float pp[3], pm[9];
    geom_pose(c, g1, pp, pm);
    float n[3] = {pm[2], pm[5], pm[8]};
    for (int k = 0; k < 3; k++) o.n[k] = n[k];
    if (t2 == DXG_BOX) {
      st.plane_box++;
      float bp[3], bm[9];
      geom_pose(c, g2, bp, bm);
      const float sz[3] = {m.geom_size[3 * g2], m.geom_size[3 * g2 + 1], m.geom_size[3 * g2 + 2]};
      float rel[3];
      sub3(rel, bp, pp);
      float cdist = dot3(rel, n);
      float ext = 0;
      for (int k = 0; k < 3; k++) ext += fabsf(bm[k] * n[0] + bm[3 + k] * n[1] + bm[6 + k] * n[2]) * sz[k];
      if (cdist > margin + ext) return 0;
      // keep the first 4 corners (in corner order) within the margin: the group's lanes
      // test corners SL, SL + NPG, ...; lane k < 4 then emits the k-th such corner
      auto corner = [&](int i, float* v) {
        float s0 = (i & 1) ? sz[0] : -sz[0], s1 = (i & 2) ? sz[1] : -sz[1], s2 = (i & 4) ? sz[2] : -sz[2];
        for (int k = 0; k < 3; k++) v[k] = bp[k] + bm[3 * k] * s0 + bm[3 * k + 1] * s1 + bm[3 * k + 2] * s2;
        float r[3];
        sub3(r, v, pp);
        return dot3(r, n);
      };
      unsigned cm = 0;  // corners within the margin, bit i = corner i
#pragma unroll
      for (int r8 = 0; r8 < 8 / NPG; r8++) {
        float v[3];
        const bool hit = corner(SL + NPG * r8, v) <= margin;
        cm |= (unsigned)((__ballot(hit) >> GBASE) & ((1ull << NPG) - 1ull)) << (NPG * r8);
      }
      const int nh = __popc(cm);
      int ik = 0, seen = 0;  // the SL-th set corner
#pragma unroll
      for (int b = 0; b < 8; b++) {
        const bool on = (cm >> b) & 1u;
        ik = (on && seen == SL) ? b : ik;
        seen += on;
      }
      float v[3];
      const float dist = corner(ik, v);
      o.wr = SL < min(4, nh);
      o.rank = SL;
      o.dist = dist;
      for (int k = 0; k < 3; k++) o.pos[k] = v[k] - 0.5f * dist * n[k];
      return min(4, nh);
    }
    st.plane_convex++;
    Shape s;
    make_shape(c, g2, 0, s);
    float nd[3] = {-n[0], -n[1], -n[2]};
    float sp[3];
    support_grp<NPG>(s, nd, sp);
    float r[3];
    sub3(r, sp, pp);
    float dist = dot3(r, n);
    if (dist > margin) return 0;
    o.wr = SL == 0;
    o.dist = dist;
    for (int k = 0; k < 3; k++) o.pos[k] = sp[k] - 0.5f * dist * n[k];
    return 1;
  }
  if (t1 == DXG_CAPSULE && t2 == DXG_CAPSULE) {
    st.capsule++;
    float p1[3], m1[9], p2[3], m2[9];
    geom_pose(c, g1, p1, m1);
    geom_pose(c, g2, p2, m2);
    float r1 = m.geom_size[3 * g1], h1 = m.geom_size[3 * g1 + 1];
    float r2 = m.geom_size[3 * g2], h2 = m.geom_size[3 * g2 + 1];
    float a1[3] = {m1[2] * h1, m1[5] * h1, m1[8] * h1}, a2[3] = {m2[2] * h2, m2[5] * h2, m2[8] * h2};
    float dv[3];
    sub3(dv, p1, p2);
    float ma = dot3(a1, a1), mb = -dot3(a1, a2), mc = dot3(a2, a2);
    float u = -dot3(a1, dv), v = dot3(a2, dv);
    float det = ma * mc - mb * mb;
    float s = 0, t = 0;
    if (det > 1e-12f) { s = (u * mc - mb * v) / det; t = (ma * v - mb * u) / det; }
    for (int it = 0; it < 3; it++) {
      s = fminf(1.f, fmaxf(-1.f, s));
      t = (v - mb * s) / fmaxf(mc, 1e-12f);
      t = fminf(1.f, fmaxf(-1.f, t));
      s = (u - mb * t) / fmaxf(ma, 1e-12f);
      s = fminf(1.f, fmaxf(-1.f, s));
    }
    float q1[3], q2[3], diff[3];
    for (int k = 0; k < 3; k++) { q1[k] = p1[k] + s * a1[k]; q2[k] = p2[k] + t * a2[k]; }
    sub3(diff, q2, q1);
    float len = norm3(diff);
    float dist = len - r1 - r2;
    if (dist > margin) return 0;
    float n[3];
    if (len > 1e-20f) { n[0] = diff[0] / len; n[1] = diff[1] / len; n[2] = diff[2] / len; }
    else { n[0] = 1; n[1] = 0; n[2] = 0; }
    o.wr = SL == 0;
    o.dist = dist;
    for (int k = 0; k < 3; k++) { o.n[k] = n[k]; o.pos[k] = q1[k] + n[k] * (r1 + 0.5f * dist); }
    return 1;
  }
  return 0;
}

// 3. narrowphase.  The wave's DX_WAVE / NPG lane groups walk the candidate list in one
// loop, each taking the next unassigned candidate when its pair is done, so a group
// never waits for another group's pair.  Contacts are written unordered together with
// their key (candidate, rank); collision() puts them into candidate order, which gives
// the list of the serial loop.  Returns the contact count (before the DX_NCON_MAX cap).
template <int NPG, class Ctx>
__device__ __forceinline__ int narrow_pass(const Ctx& c, int ng, const int* gcand, const float4* gcrec, float* con,
                                           int* cntq) {
  int ncon = 0;
  NpStats st = {0, 0, 0, 0, 0, 0, 0};
  {
    const int grp = LANE / NPG;
    int q = grp, next = DX_WAVE / NPG;
    bool fresh = true;
    int gp = 0;
    float margin = 0;
    Shape G;  // the pair's first geom on the group's first half of lanes, its second on the other
    MprState M;
    bool cached = false;
    int trips = 0;
    M.P = c.f(c.L.cand + c.L.cand_max) + MP_WORDS * grp;  // free during collision (dx_api.hip layout)
    const NpClock ck{c.stage_acc, c.I};
    for (;;) {
      bool act = q < ng;
      if (__ballot(act) == 0) break;
      trips++;
      ck.mark(ST_NP_LOOP);

      NpOut o;
      o.wr = false;
      o.rank = 0;
      int cnt = 0;
      bool done = false;
      if (act) {
        bool stepping = !fresh;
        if (fresh) {
          gp = gcand[q];
          const float4 pr = gcrec[q];
          if (__float_as_int(pr.w)) {
            cnt = narrowphase_prim<NPG>(c, gp, o, st);
            done = true;
          } else {
            st.mpr++;
            margin = pr.z;
            make_shape_rec(c, __float_as_int(half_b<NPG>() ? pr.y : pr.x), 0.5f * margin, G);
            float4 ce = c.sep ? c.sep[gp & (DX_SEP_SLOTS - 1)] : make_float4(0.f, 0.f, 0.f, 0.f);
            cached = __float_as_int(ce.w) == gp + 1;
            const float cd[3] = {ce.x, ce.y, ce.z};
            mpr_init<NPG>(G, M, cached ? cd : nullptr);
            fresh = false;
            stepping = true;
          }
        }
        ck.mark(ST_NP_FRESH);
        if (stepping) {
          float depth, nrm[3], pos[3];
          int r = mpr_step<NPG>(G, M, depth, nrm, pos, st, ck);
          ck.mark(ST_NP_PORTAL);
          if (r && c.sep && SL == 0) {
            // remember a separating direction (unless it is the cached one, still
            // separating: phase -1); forget it once the pair touches.  Plain stores: an
            // entry decides a verdict only where MPR's own verdict is the same (mpr_init,
            // DX_SEP_CLEAR), so a task on another XCD that reads an older entry (its L2
            // has not seen this one), or a layout that gives the slot to the other pair
            // sharing it, computes the same contacts; written through (DX_SEP_WT) every
            // 16-B entry cost a partial-line HBM write and the next task's read a miss.
            const bool keep = r == 1 && M.phase != -1;
            if (keep || (cached && (r == 2 || !DX_SEP_KEEP))) {
              const float4 ent = keep ? make_float4(M.dir[0], M.dir[1], M.dir[2], __int_as_float(gp + 1))
                                      : make_float4(0.f, 0.f, 0.f, 0.f);
              if (DX_SEP_WT) st_sc1_f4(c.sep, 16 * DX_SEP_SLOTS, 16 * (gp & (DX_SEP_SLOTS - 1)), ent);
              else c.sep[gp & (DX_SEP_SLOTS - 1)] = ent;
            }
          }
          if (r) {
            done = true;
            if (r == 2) {
              st.hit++;
              cnt = 1;
              o.wr = SL == 0;
              o.dist = margin - depth;
              for (int k = 0; k < 3; k++) { o.n[k] = nrm[k]; o.pos[k] = pos[k]; }
            }
          }
        }
      }
      if (__ballot(cnt > 0)) {  // most loop trips produce no contact
        // contacts of the groups before this one (cnt is uniform within a group)
        const int cinc = wave_incl_scan(SL == 0 ? cnt : 0);
        const int pre = __shfl(cinc, GBASE, 64) - cnt;
        int slot = ncon + pre + o.rank;
        if (o.wr && slot < DX_NCON_MAX + DX_NCON_SPARE) {
          write_contact(con, slot, o.pos, o.n, o.dist, gp);
          con[DX_CON_STRIDE * slot + 14] = __int_as_float(4 * q + o.rank);  // sort key
        }
        ncon += __builtin_amdgcn_readlane(cinc, 63);
      }
      // a group that finished its pair takes the next unassigned candidate (in group
      // order), so a long MPR on one group no longer holds back the others' queues;
      // the contact keys still sort the list into candidate order below
      const uint64_t fin = __ballot(done && SL == 0);
      if (done && SL == 0) cntq[q] = cnt;  // contacts of candidate q (the pool cut, collision())
      if (done) {
        q = next + __popcll(fin & ((1ull << GBASE) - 1ull));
        fresh = true;
      }
      next += __popcll(fin);
    }
    stage_count(c, CNT_NP_TRIPS, trips);
  }
  SYNC();
  if (c.stage_acc) {
    bool lead = SL == 0;
    int v[7] = {st.plane_box, st.plane_convex, st.capsule, st.mpr, st.support, st.hit, st.maxit};
#pragma unroll
    for (int k = 0; k < 7; k++) stage_count(c, CNT_PLANE_BOX + k, wave_sum_i(lead ? v[k] : 0));
  }
  return ncon;
}

// broadphase (body spheres, lanes over body pairs) -> flattened mid-phase (geom
// spheres, lanes over every geom pair of the surviving body pairs) -> narrowphase
// (whole wave per pair).  Writes contact records into LDS.
// watch_only: only pairs containing geom `wg` and a geom of body `wb` (observation pass).
template <class Ctx>
__device__ __forceinline__ void collision(const Ctx& c, int watch_only, int wg, int wb, const int* wlist = nullptr,
                                          int wn = 0) {
  const DevModel& m = c.mdl();
  int* I = c.I;
  int* cand = (int*)c.f(c.L.cand);
  int cmax = c.L.cand_max;
  if (LANE == 0) { I[I_NCON] = 0; I[I_NCAND] = 0; }
  SYNC();
  if (c.disable_contact) return;
  float* xpos = c.f(c.L.xpos);
  float* xmat = c.f(c.L.xmat);
  // 1. body-pair cull -> cand[0..nbc) body-pair ids, pref[0..nbc] prefix of geom-pair counts.
  // Bounding spheres (and planes) over all body pairs, lane per pair; the survivors go
  // to a list, and one pass over the list applies the box test (dx_api.hip bpair_rec)
  // and compacts: the box SAT then runs on ~1 chunk of survivors, not on every chunk.
  int half = cmax / 3;
  int* pref = cand + half;
  int nbc = 0, ngp = 0;
  int* sl = (int*)(c.f(c.L.cand + c.L.cand_max) + DX_NGRP_MAX * MP_WORDS);  // the pair-record area, unused yet
  const int slcap = 4 * (cmax - 2 * half);
  int nsl = 0;
  auto flush = [&]() {
    for (int b0 = 0; b0 < nsl; b0 += DX_WAVE) {
      const int k = b0 + LANE;
      bool keep = false;
      int cnt = 0, adr = 0;
      if (k < nsl) {
        const int e = sl[k];
        const DXG float4* R = m.bpair_rec + 7 * (e & 0x7fffffff);
        const float4 r0 = R[0], r3 = R[3], r4 = R[4], r5 = R[5], r6 = R[6];
        keep = true;
        if (e < 0) {  // sphere-tested pair: boxes around its geoms' OBBs
          const int b1 = __float_as_int(r0.x), b2 = __float_as_int(r0.y);
          const float b1c[3] = {r4.x, r4.y, r4.z}, b1e[3] = {r4.w, r5.x, r5.y};
          const float b2c[3] = {r5.z, r5.w, r6.x}, b2e[3] = {r6.y, r6.z, r6.w};
          keep = box_overlap(b1c, b1e, xpos + 3 * b1, xmat + 9 * b1, b2c, b2e, xpos + 3 * b2, xmat + 9 * b2, r3.w);
        }
        adr = __float_as_int(r0.z);
        cnt = keep ? __float_as_int(r0.w) : 0;
      }
      uint64_t mask = __ballot(keep);
      int pos = __popcll(mask & ((1ull << LANE) - 1ull));
      int inc = wave_incl_scan(cnt);
      int off = inc - cnt;
      if (keep && nbc + pos < half) {
        cand[nbc + pos] = adr;  // first geom pair of the body pair
        pref[nbc + pos] = ngp + off;
      }
      nbc += __popcll(mask);
      ngp += __builtin_amdgcn_readlane(inc, 63);
    }
    nsl = 0;
    SYNC();
  };
  // the next chunk's records are loaded while this chunk is tested (one memory
  // round trip in flight across chunk boundaries)
  float4 nx[6];
  // the observation pass's watch test walks only the body pairs that can hold the
  // watched contact (dx_set_watch builds that list on the host)
  const int nloop = (watch_only && wlist) ? wn : c.nbpair;
  auto bpidx = [&](int i) { return (watch_only && wlist) ? wlist[i] : i; };
  {
    const int i0 = max(min(LANE, nloop - 1), 0);
    const DXG float4* R = m.bpair_rec + 7 * (nloop > 0 ? bpidx(i0) : 0);
#pragma unroll
    for (int k = 0; k < 6; k++) nx[k] = R[k];
  }
  for (int base = 0; base < nloop; base += DX_WAVE) {
    const int bp = base + LANE < nloop ? bpidx(base + LANE) : c.nbpair;
    bool keep = false, box = false;
    const float4 r0 = nx[0], s1 = nx[1], s2 = nx[2], r3 = nx[3], r4 = nx[4], r5 = nx[5];
    if (base + DX_WAVE < nloop) {
      const DXG float4* R = m.bpair_rec + 7 * bpidx(min(base + DX_WAVE + LANE, nloop - 1));
#pragma unroll
      for (int k = 0; k < 6; k++) nx[k] = R[k];
    }
    if (bp < c.nbpair) {
      int b1 = __float_as_int(r0.x), b2 = __float_as_int(r0.y);
      keep = true;
      if (watch_only) keep = (b2 == wb || b1 == wb) && (m.geom_bodyid[wg] == b1 || m.geom_bodyid[wg] == b2);
      float mg = r3.x;
      int pg = __float_as_int(r3.y);
      if (keep && s2.w >= 0) {
        float c2[3];
        const float s2v[3] = {s2.x, s2.y, s2.z};
        matvec3(c2, xmat + 9 * b2, s2v);
        for (int k = 0; k < 3; k++) c2[k] += xpos[3 * b2 + k];
        if (pg >= 0) {
          int pb = __float_as_int(r3.z);
          const float pl[3] = {r4.x, r4.y, r4.z}, nl[3] = {r5.x, r5.y, r5.z};
          float pp[3], n[3];
          matvec3(pp, xmat + 9 * pb, pl);
          matvec3(n, xmat + 9 * pb, nl);
          float rr[3] = {c2[0] - pp[0] - xpos[3 * pb], c2[1] - pp[1] - xpos[3 * pb + 1], c2[2] - pp[2] - xpos[3 * pb + 2]};
          keep = dot3(rr, n) <= s2.w + mg;
        } else if (s1.w >= 0) {
          float c1[3];
          const float s1v[3] = {s1.x, s1.y, s1.z};
          matvec3(c1, xmat + 9 * b1, s1v);
          for (int k = 0; k < 3; k++) c1[k] += xpos[3 * b1 + k];
          keep = sphere_overlap(c1, s1.w, c2, s2.w, mg);
          box = true;
        }
      }
    }
    uint64_t mask = __ballot(keep);
    int pos = __popcll(mask & ((1ull << LANE) - 1ull));
    if (keep) sl[nsl + pos] = box ? (bp | (int)0x80000000) : bp;
    nsl += __popcll(mask);
    SYNC();
    if (nsl > slcap - DX_WAVE) flush();
  }
  flush();
  if (nbc > half) { nbc = half; if (LANE == 0) I[I_OVF] |= 1; }
  if (LANE == 0) pref[nbc] = ngp;
  SYNC();
  stage_mark(c, ST_BROAD);
  // 2. flattened geom-pair mid-phase: lane t -> (body pair q, geom pair) by binary search
  int* gcand = pref + half;
  int gmax = cmax - 2 * half;
  // pair records of the surviving candidates, after the four groups' portal points
  // (dx_api.hip layout reserves 4 * gmax words there)
  float4* gcrec = (float4*)(c.f(c.L.cand + c.L.cand_max) + DX_NGRP_MAX * MP_WORDS);
  int ng = 0;
  int total = nbc > 0 ? pref[nbc] : 0;
  for (int base = 0; base < total; base += DX_WAVE) {
    int t = base + LANE;
    bool keep = false;
    int gp = -1;
    float4 prec = make_float4(0.f, 0.f, 0.f, 0.f);
    if (t < total) {
      int lo = 0, hi = nbc;  // pref[lo] <= t < pref[hi]
      while (hi - lo > 1) {
        int mid = (lo + hi) >> 1;
        if (pref[mid] <= t) lo = mid; else hi = mid;
      }
      gp = cand[lo] + (t - pref[lo]);
      float4 pr = m.gpair_rec[gp];
      prec = pr;
      int g1 = __float_as_int(pr.x), g2 = __float_as_int(pr.y);
      keep = !watch_only || g1 == wg || g2 == wg;
      if (keep) {
        float mg = pr.z;
        const DXG float4* G1 = m.geom_crec + 6 * g1;
        const DXG float4* G2 = m.geom_crec + 6 * g2;
        float4 a0 = G1[0], a1 = G1[1], a2 = G1[2], a3 = G1[3], a4 = G1[4], a5 = G1[5];
        float4 e0 = G2[0], e1 = G2[1], e2 = G2[2], e3 = G2[3], e4 = G2[4], e5 = G2[5];
        int b1 = __float_as_int(a0.y), b2 = __float_as_int(e0.y);
        float c2[3];
        const float s2[3] = {e1.x, e1.y, e1.z};
        matvec3(c2, xmat + 9 * b2, s2);
        for (int k = 0; k < 3; k++) c2[k] += xpos[3 * b2 + k];
        if (__float_as_int(a0.x) == DXG_PLANE) {
          const float pl[3] = {a2.x, a2.y, a2.z}, nl[3] = {a5.x, a5.y, a5.z};
          float p1[3], n[3], r[3];
          matvec3(p1, xmat + 9 * b1, pl);
          matvec3(n, xmat + 9 * b1, nl);
          for (int k = 0; k < 3; k++) r[k] = c2[k] - p1[k] - xpos[3 * b1 + k];
          keep = dot3(r, n) <= e1.w + mg;
        } else {
          const float s1[3] = {a1.x, a1.y, a1.z};
          float c1[3];
          matvec3(c1, xmat + 9 * b1, s1);
          for (int k = 0; k < 3; k++) c1[k] += xpos[3 * b1 + k];
          keep = sphere_overlap(c1, a1.w, c2, e1.w, mg);
          if (keep) {
            const float o1[15] = {a2.x, a2.y, a2.z, a2.w, a3.x, a3.y, a3.z, a3.w, a4.x, a4.y, a4.z, a4.w, a5.x, a5.y, a5.z};
            const float o2[15] = {e2.x, e2.y, e2.z, e2.w, e3.x, e3.y, e3.z, e3.w, e4.x, e4.y, e4.z, e4.w, e5.x, e5.y, e5.z};
            keep = obb_overlap(o1, xpos + 3 * b1, xmat + 9 * b1, o2, xpos + 3 * b2, xmat + 9 * b2, mg);
          }
        }
      }
    }
    uint64_t mask = __ballot(keep);
    int pos = __popcll(mask & ((1ull << LANE) - 1ull));
    if (keep && ng + pos < gmax) {
      gcand[ng + pos] = gp;
      gcrec[ng + pos] = prec;  // the narrowphase reads the pair record from LDS
    }
    ng += __popcll(mask);
  }
  if (ng > gmax) {
    if (LANE == 0) I[I_OVF] |= 1;
    ng = gmax;
  }
  if (LANE == 0) I[I_NCAND] = ng;
  stage_count(c, CNT_BROAD_KEEP, nbc);
  stage_count(c, CNT_MID_PAIRS, total);
  stage_count(c, CNT_MID_KEEP, ng);
  SYNC();
  stage_mark(c, ST_MID);
  // 3. narrowphase (narrow_pass): eight pairs per wave, or sixteen (four-lane groups)
  // when the substep has more than eight candidates -- the contact-rich states whose
  // serial chains of pairs per group bound the heaviest environments' substeps
  float* con = c.f(c.L.con);
  int* cntq = cand;  // the body-pair list is dead now: contacts per narrowphase candidate
  const int ncon_raw = ng > c.np_wide ? narrow_pass<4>(c, ng, gcand, gcrec, con, cntq)
                                      : narrow_pass<8>(c, ng, gcand, gcrec, con, cntq);
  int ncon = ncon_raw;
  SYNC();
  if (ncon_raw > (c.defer ? min(DX_NCON_MAX, c.defer_at) : DX_NCON_MAX) && !watch_only) {
    if (c.defer) {
      // the step kernel's pool is full: this physics step runs in the overflow tier
      // (dx_step_hi, DX_NCON_HI contacts) from the unchanged state (env_substep)
      if (LANE == 0) { I[I_DEFER] = 1; I[I_NRAW] = max(I[I_NRAW], ncon_raw); }
      SYNC();
      return;
    }
    // The pool keeps the first DX_NCON_MAX contacts in candidate (generation) order, as
    // MuJoCo fills its contact buffer: the records above were kept in completion order,
    // so the candidates up to the one whose contacts cross the cap run again with every
    // contact kept (DX_NCON_SPARE extra record slots hold the crossing candidate's), and
    // the sort and the cap below drop the rest.  (The verdicts and contacts of a rerun
    // pair are the first run's: the separating-direction cache never decides one.)
    int v[4], sum = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {  // ng <= 256 candidates: four per lane
      const int q = 4 * LANE + k;
      v[k] = q < ng ? cntq[q] : 0;
      sum += v[k];
    }
    const int ex = wave_incl_scan(sum) - sum;
    int qcut = 1 << 30, run = ex;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      run += v[k];
      qcut = (run > DX_NCON_MAX && qcut == (1 << 30)) ? 4 * LANE + k : qcut;
    }
    qcut = wave_min_i(qcut);
    SYNC();
    ncon = qcut + 1 > c.np_wide ? narrow_pass<4>(c, qcut + 1, gcand, gcrec, con, cntq)
                                : narrow_pass<8>(c, qcut + 1, gcand, gcrec, con, cntq);
    SYNC();
  }
  // candidate order: lane k ranks record k (and k + 64, ...) by its key, then moves it
  {
    constexpr int NS = (DX_NCON_MAX + DX_NCON_SPARE + DX_WAVE - 1) / DX_WAVE;
    const int nk = min(ncon, DX_NCON_MAX + DX_NCON_SPARE);
    int key[NS], rank[NS];
    float rec[NS][14];
#pragma unroll
    for (int k = 0; k < NS; k++) {
      const int i = LANE + DX_WAVE * k;
      key[k] = i < nk ? __float_as_int(con[DX_CON_STRIDE * i + 14]) : 0x7fffffff;
      rank[k] = 0;
    }
#pragma unroll
    for (int cc = 0; cc < NS; cc++) {
      const int nj = min(nk - DX_WAVE * cc, DX_WAVE);
      for (int j = 0; j < nj; j++) {
        const int kj = __builtin_amdgcn_readlane(key[cc], j);
#pragma unroll
        for (int k = 0; k < NS; k++) rank[k] += kj < key[k];
      }
    }
#pragma unroll
    for (int k = 0; k < NS; k++) {
      const int i = LANE + DX_WAVE * k;
#pragma unroll
      for (int e = 0; e < 14; e++) rec[k][e] = i < nk ? con[DX_CON_STRIDE * i + e] : 0.f;
    }
    SYNC();
#pragma unroll
    for (int k = 0; k < NS; k++) {
      if (LANE + DX_WAVE * k < nk) {
#pragma unroll
        for (int e = 0; e < 14; e++) con[DX_CON_STRIDE * rank[k] + e] = rec[k][e];
      }
    }
  }
  stage_mark(c, ST_NP_MPR);
  if (LANE == 0 && !watch_only) I[I_NRAW] = max(I[I_NRAW], ncon_raw);
  if (ncon > DX_NCON_MAX) {
    if (LANE == 0) I[I_OVF] |= 2;
    ncon = DX_NCON_MAX;
  }
  SYNC();
  if (LANE == 0) I[I_NCON] = ncon;
  SYNC();
  stage_mark(c, ST_NARROW);
}

// ------------------------------------------------------------------------ //
// constraints
// ------------------------------------------------------------------------ //
__device__ __forceinline__ float impedance(const float* solimp, float violation) {
  float d0 = fminf(0.9999f, fmaxf(0.0001f, solimp[0]));
  float dmax = fminf(0.9999f, fmaxf(0.0001f, solimp[1]));
  float width = solimp[2], mid = solimp[3], power = solimp[4];
  if (width <= 1e-15f || d0 == dmax) return 0.5f * (d0 + dmax);
  float x = fabsf(violation) / width;
  if (x >= 1) return dmax;
  float y;
  if (power == 1) y = x;
  else if (power == 2) y = x <= mid ? x * x / mid : 1 - (1 - x) * (1 - x) / (1 - mid);  // MuJoCo's default
  else if (x <= mid) y = powf(x, power) / powf(mid, power - 1);
  else y = 1 - powf(1 - x, power) / powf(1 - mid, power - 1);
  return d0 + y * (dmax - d0);
}

// row parameters -> D, aref, Rf.  vel = J*qvel.
template <class Ctx>
__device__ __forceinline__ void row_params(const Ctx& c, int r, float pos, float margin, float floss, float diag,
                           const float* solref, const float* solimp, float vel, float rscale, bool fric) {
  const DevModel& m = c.mdl();
  float imp = impedance(solimp, pos - margin);
  float tc = fmaxf(solref[0], 2 * m.timestep), dr = solref[1];
  float dmax = fminf(0.9999f, fmaxf(0.0001f, solimp[1]));
  float K = 1.0f / fmaxf(1e-15f, dmax * dmax * tc * tc * dr * dr);
  float B = 2.0f / fmaxf(1e-15f, dmax * tc);
  float R = fmaxf(1e-15f, (1 - imp) / imp * diag);
  R = fmaxf(1e-15f, R * rscale);
  c.f(c.L.efc_D)[r] = 1.0f / R;
  if (fric) {  // friction rows come first: efc_fl / efc_Rf hold only [0, nfric)
    c.f(c.L.efc_fl)[r] = floss;
    c.f(c.L.efc_Rf)[r] = R * floss;
  }
  float viol = fric ? 0.f : pos - margin;
  c.f(c.L.efc_aref)[r] = -B * vel - K * imp * viol;
}

// sparse contact jacobian (frame rows) -> cj_idx / cj_val; then all rows
template <class Ctx>
__device__ __forceinline__ void make_constraint(const Ctx& c) {
  const DevModel& m = c.mdl();
  int nv = c.nv;
  int* I = c.I;
  float* qpos = c.f(c.L.qpos);
  float* qvel = c.f(c.L.qvel);
  int* meta = (int*)c.f(c.L.efc_meta);
  int nfric = c.nfric;
  float* con = c.f(c.L.con);
  // Model tables of every section's first lane pass (lane = friction row, limited joint,
  // contact), issued up front in dependency levels: three overlapped L2 round trips
  // instead of a chain of them per section after each barrier.
  // level 1
  const int ncon = I[I_NCON];
  const bool fok = LANE < nfric, lok = LANE < c.nlimj;
  bool cok = LANE < ncon;
  const int fd = fok ? m.fric_dof[LANE] : 0;
  const int lj = lok ? m.limj_jnt[LANE] : 0;
  // (contact tables only for lanes holding a contact: a scene without contact pairs
  // has empty gpair tables)
  int cgp = cok ? __float_as_int(con[DX_CON_STRIDE * LANE + 13]) : 0;
  int cg1 = cok ? m.gpair_geom[2 * cgp] : 0, cg2 = cok ? m.gpair_geom[2 * cgp + 1] : 0;
  int ccd = cok ? m.gpair_condim[cgp] : 1;
  float cfr0 = cok ? m.gpair_friction[5 * cgp] : 0.f, cfr1 = cok ? m.gpair_friction[5 * cgp + 1] : 0.f;
  float csr[2] = {cok ? m.gpair_solref[2 * cgp] : 0.f, cok ? m.gpair_solref[2 * cgp + 1] : 0.f};
  float csi[5];
  for (int e = 0; e < 5; e++) csi[e] = cok ? m.gpair_solimp[5 * cgp + e] : 0.f;
  float cmg = cok ? m.gpair_margin[cgp] : 0.f;
  // level 2
  const float ffl = m.dof_frictionloss[fd], fiw = m.dof_invweight0[fd];
  const float fsr[2] = {m.dof_solref[2 * fd], m.dof_solref[2 * fd + 1]};
  float fsi[5];
  for (int e = 0; e < 5; e++) fsi[e] = m.dof_solimp[5 * fd + e];
  const int lqa = m.jnt_qposadr[lj], ldof = m.jnt_dofadr[lj];
  const float lr0 = m.jnt_range[2 * lj], lr1 = m.jnt_range[2 * lj + 1], lmg = m.jnt_margin[lj];
  const float lsr[2] = {m.jnt_solref[2 * lj], m.jnt_solref[2 * lj + 1]};
  float lsi[5];
  for (int e = 0; e < 5; e++) lsi[e] = m.jnt_solimp[5 * lj + e];
  int cb1 = cok ? m.geom_bodyid[cg1] : 0, cb2 = cok ? m.geom_bodyid[cg2] : 0;
  // level 3
  const float liw = m.dof_invweight0[ldof];
  uint64_t cc1 = m.body_chain[cb1], cc2 = m.body_chain[cb2];
  float ctran = m.body_invweight0[2 * cb1] + m.body_invweight0[2 * cb2];
  int cr1 = m.body_rootidx[cb1], cr2 = m.body_rootidx[cb2];
  // 1. dof friction rows: fixed positions [0, nfric)
  for (int k = LANE; k < nfric; k += DX_WAVE) {
    const bool own = k == LANE;
    int d = own ? fd : m.fric_dof[k];
    meta[k] = DXR_FRIC | (d << 8);
    if (own)
      row_params(c, k, 0, 0, ffl, fiw, fsr, fsi, qvel[d], 1.0f, true);
    else
      row_params(c, k, 0, 0, m.dof_frictionloss[d], m.dof_invweight0[d], m.dof_solref + 2 * d,
                 m.dof_solimp + 5 * d, qvel[d], 1.0f, true);
  }
  // 2. joint limits (one side at most unless range < 2 margin): lane per limited joint
  int nrow = nfric;
  for (int base = 0; base < c.nlimj; base += DX_WAVE) {
    int k = base + LANE;
    int cnt = 0;
    float dist[2];
    int j = -1;
    const bool own = base == 0;  // first pass: the preloaded tables
    float mg = 0.f;
    if (k < c.nlimj) {
      j = own ? lj : m.limj_jnt[k];
      float q = qpos[own ? lqa : m.jnt_qposadr[j]];
      dist[0] = q - (own ? lr0 : m.jnt_range[2 * j]);
      dist[1] = (own ? lr1 : m.jnt_range[2 * j + 1]) - q;
      mg = own ? lmg : m.jnt_margin[j];
      cnt = (dist[0] < mg) + (dist[1] < mg);
    }
    int inc = wave_incl_scan(cnt);
    int off = inc - cnt;
    int tot = __builtin_amdgcn_readlane(inc, 63);
    if (cnt) {
      int r = nrow + off;
      int d = own ? ldof : m.jnt_dofadr[j];
      for (int side = 0; side < 2; side++) {
        if (dist[side] >= mg) continue;
        if (r < c.L.nefc_max) {
          meta[r] = DXR_LIMJ | (side << 4) | (d << 8);  // hinge: the joint's dof
          float v = side == 0 ? qvel[d] : -qvel[d];
          if (own)
            row_params(c, r, dist[side], mg, 0, liw, lsr, lsi, v, 1.0f, false);
          else
            row_params(c, r, dist[side], mg, 0, m.dof_invweight0[d], m.jnt_solref + 2 * j,
                       m.jnt_solimp + 5 * j, v, 1.0f, false);
        }
        r++;
      }
    }
    nrow += tot;
  }
  // 3. tendon limits
  float* tl = c.f(c.L.ten_len);
  for (int base = 0; base < c.nlimt; base += DX_WAVE) {
    int k = base + LANE;
    int cnt = 0;
    float dist[2];
    int t = -1;
    if (k < c.nlimt) {
      t = m.limt_ten[k];
      dist[0] = tl[t] - m.tendon_range[2 * t];
      dist[1] = m.tendon_range[2 * t + 1] - tl[t];
      cnt = (dist[0] < m.tendon_margin[t]) + (dist[1] < m.tendon_margin[t]);
    }
    int inc = wave_incl_scan(cnt);
    int off = inc - cnt;
    int tot = __builtin_amdgcn_readlane(inc, 63);
    if (cnt) {
      int r = nrow + off;
      float tv = 0;
      for (int w = m.tendon_adr[t]; w < m.tendon_adr[t] + m.tendon_num[t]; w++)
        tv += m.wrap_coef[w] * qvel[m.wrap_dof[w]];
      for (int side = 0; side < 2; side++) {
        if (dist[side] >= m.tendon_margin[t]) continue;
        if (r < c.L.nefc_max) {
          meta[r] = DXR_LIMT | (side << 4) | (t << 8);
          row_params(c, r, dist[side], m.tendon_margin[t], 0, m.tendon_invweight0[t],
                     m.tendon_solref + 2 * t, m.tendon_solimp + 5 * t, side == 0 ? tv : -tv, 1.0f, false);
        }
        r++;
      }
    }
    nrow += tot;
  }
  SYNC();
  // 4. contacts: sparse frame jacobian, then pyramid rows, in chunks of DX_WAVE contacts
  // (one chunk for DX_NCON_MAX <= 64 -- the step kernel; the overflow tier's larger pool
  // takes several).  Lane = contact of the chunk for the support masks and record fields
  // (chunk 0's tables were loaded above); then the Jacobian entries flattened over
  // (contact, support dof) items -- every item one lane, no serial walk over a contact's
  // dofs -- and the frame velocities J qvel as jac_vec's gather.
  float* cdof = c.f(c.L.cdof);
  float* rcom = c.f(c.L.rcom);
  unsigned char* cj_idx = (unsigned char*)c.f(c.L.cj_idx);
  float* cj_val = c.f(c.L.cj_val);
  float* cq = c.f(c.L.cq);
  constexpr int NCH = DX_NCH;
#pragma unroll 1
  for (int ch = 0; ch < NCH; ch++) {
    const int cb = ch * DX_WAVE;
    if (cb >= ncon) break;  // uniform
    const int nc = min(ncon - cb, DX_WAVE);  // contacts in this chunk
    if (ch > 0) {  // (overflow tier only) this chunk's tables
      const int ci = cb + LANE;
      cok = ci < ncon;
      cgp = cok ? __float_as_int(con[DX_CON_STRIDE * ci + 13]) : 0;
      cg1 = cok ? m.gpair_geom[2 * cgp] : 0;
      cg2 = cok ? m.gpair_geom[2 * cgp + 1] : 0;
      ccd = cok ? m.gpair_condim[cgp] : 1;
      cfr0 = cok ? m.gpair_friction[5 * cgp] : 0.f;
      cfr1 = cok ? m.gpair_friction[5 * cgp + 1] : 0.f;
      csr[0] = cok ? m.gpair_solref[2 * cgp] : 0.f;
      csr[1] = cok ? m.gpair_solref[2 * cgp + 1] : 0.f;
      for (int e = 0; e < 5; e++) csi[e] = cok ? m.gpair_solimp[5 * cgp + e] : 0.f;
      cmg = cok ? m.gpair_margin[cgp] : 0.f;
      cb1 = cok ? m.geom_bodyid[cg1] : 0;
      cb2 = cok ? m.geom_bodyid[cg2] : 0;
      cc1 = m.body_chain[cb1];
      cc2 = m.body_chain[cb2];
      ctran = m.body_invweight0[2 * cb1] + m.body_invweight0[2 * cb2];
      cr1 = m.body_rootidx[cb1];
      cr2 = m.body_rootidx[cb2];
    }
    int nnz = 0;
    const uint64_t sp = cok ? cc1 ^ cc2 : 0ull;
    if (cok) {
      float* r = con + DX_CON_STRIDE * (cb + LANE);
      const int np = __popcll(sp);
      nnz = min(np, DX_DOFMAX);
      if (np > DX_DOFMAX) I[I_OVF] |= 4;
      r[14] = __int_as_float(nnz | ((ccd == 1 ? 1 : 4) << 8));
      r[16] = cfr0;
      r[17] = cfr1;
      r[18] = __int_as_float((int)(uint32_t)sp);
      r[19] = __int_as_float((int)(uint32_t)(sp >> 32));
    }
    {
      const int incl = wave_incl_scan(nnz);
      const int excl = incl - nnz;
      const int total = __builtin_amdgcn_readlane(incl, 63);
      const unsigned splo = (unsigned)sp, sphi = (unsigned)(sp >> 32);
      const unsigned c1lo = (unsigned)cc1, c1hi = (unsigned)(cc1 >> 32);
      const unsigned c2lo = (unsigned)cc2, c2hi = (unsigned)(cc2 >> 32);
      for (int base = 0; base < total; base += DX_WAVE) {  // uniform trip count: the shuffles see every lane
        const int t = min(base + LANE, total - 1);
        int ci = 0;  // last contact (of the chunk) whose first item is <= t
#pragma unroll
        for (int st = DX_SEARCH0; st >= 1; st >>= 1) {
          const int mid = ci + st;
          const int em = __shfl(excl, mid & 63, 64);
          if (mid < nc && em <= t) ci = mid;
        }
        int q = t - __shfl(excl, ci, 64);
        const int slot = q;
        // the q-th set bit of the contact's support mask: 32-bit half, then halving
        // windows by popcount
        const unsigned lo = (unsigned)__shfl((int)splo, ci, 64), hi = (unsigned)__shfl((int)sphi, ci, 64);
        const int plo = __popc(lo);
        unsigned w = q < plo ? lo : hi;
        int d = q < plo ? 0 : 32;
        q = q < plo ? q : q - plo;
#pragma unroll
        for (int h = 16; h >= 1; h >>= 1) {
          const unsigned low = w & ((1u << h) - 1u);
          const int pc = __popc(low);
          const bool up = q >= pc;
          q = up ? q - pc : q;
          w = up ? (w >> h) : low;
          d += up ? h : 0;
        }
        // (every shuffle unconditional: a shuffle under a divergent select would read
        // inactive source lanes)
        const unsigned a1l = (unsigned)__shfl((int)c1lo, ci, 64), a1h = (unsigned)__shfl((int)c1hi, ci, 64);
        const unsigned a2l = (unsigned)__shfl((int)c2lo, ci, 64), a2h = (unsigned)__shfl((int)c2hi, ci, 64);
        const int t1 = __shfl(cr1, ci, 64), t2 = __shfl(cr2, ci, 64);
        const unsigned b1 = d < 32 ? a1l >> d : a1h >> (d - 32);
        const unsigned b2 = d < 32 ? a2l >> d : a2h >> (d - 32);
        const int rt = (b1 & 1u) ? t1 : t2;
        const float sgn = (b2 & 1u) ? 1.f : -1.f;
        const int cg = cb + ci;
        const float* r = con + DX_CON_STRIDE * cg;
        const float* rc = rcom + 3 * rt;
        const float* cd = cdof + 6 * d;
        const float off[3] = {r[0] - rc[0], r[1] - rc[1], r[2] - rc[2]};
        float tq[3];
        cross3(tq, cd, off);
        const float jp[3] = {cd[3] + tq[0], cd[4] + tq[1], cd[5] + tq[2]};
        if (base + LANE < total) {
          cj_idx[cg * DX_DOFMAX + slot] = (unsigned char)d;
#pragma unroll
          for (int k = 0; k < 3; k++)
            cj_val[(cg * 3 + k) * DX_DOFMAX + slot] = sgn * (r[3 + 3 * k] * jp[0] + r[4 + 3 * k] * jp[1] + r[5 + 3 * k] * jp[2]);
        }
      }
    }
    SYNC();
    // frame velocities (J qvel), lane = (contact, frame axis)
    for (int t = 3 * cb + LANE; t < 3 * (cb + nc); t += DX_WAVE) {
      const int ci = t / 3, k = t - 3 * ci;
      const int nz = __float_as_int(con[DX_CON_STRIDE * ci + 14]) & 255;
      float v = 0;
#pragma unroll
      for (int q = 0; q < DX_DOFMAX; q++) {  // unguarded loads; slots past nnz are not summed
        const float jv = cj_val[(ci * 3 + k) * DX_DOFMAX + q];
        const float xv = qvel[cj_idx[ci * DX_DOFMAX + q]];
        const float tt = v + jv * xv;
        v = q < nz ? tt : v;
      }
      cq[t] = v;
    }
    SYNC();
    // pyramid rows, lane = contact of the chunk (its tables loaded above)
    {
      const int ci = cb + LANE;
      int nr = 0;
      float* r = nullptr;
      if (LANE < nc) {
        r = con + DX_CON_STRIDE * ci;
        nr = __float_as_int(r[14]) >> 8;
      }
      int inc = wave_incl_scan(nr);
      int off = inc - nr;
      int tot = __builtin_amdgcn_readlane(inc, 63);
      if (nr) {
        r[15] = __int_as_float(nrow + off);
        if (nr == 1) {
          int row = nrow + off;
          if (row < c.L.nefc_max) {
            meta[row] = DXR_CONFL | (ci << 8);
            row_params(c, row, r[12], cmg, 0, ctran, csr, csi, cq[3 * ci], 1.0f, false);
          }
        } else {
          float rs = 2 * cfr0 * cfr0 / m.impratio;
          for (int e = 0; e < 4; e++) {
            int row = nrow + off + e;
            if (row >= c.L.nefc_max) break;
            int k = 1 + (e >> 1);
            float mu = (k == 1 ? cfr0 : cfr1) * ((e & 1) ? -1.f : 1.f);
            meta[row] = DXR_CON | (e << 4) | (ci << 8);
            row_params(c, row, r[12], cmg, 0, ctran, csr, csi, cq[3 * ci] + mu * cq[3 * ci + k], rs, false);
          }
        }
      }
      nrow += tot;
    }
  }
  if (nrow > c.L.nefc_max) {
    if (LANE == 0) I[I_OVF] |= 8;
    nrow = c.L.nefc_max;
  }
  if (LANE == 0) I[I_NEFC] = nrow;
  SYNC();
}

// ------------------------------------------------------------------------ //
// velocity stage: comVel, RNE (+ applied wrench), passive, actuation
// ------------------------------------------------------------------------ //
template <class Ctx>
__device__ __forceinline__ void velocity_stage(const Ctx& c, const float* xfrc) {
  const DevModel& m = c.mdl();
  int nv = c.nv;
  float* qvel = c.f(c.L.qvel);
  float* cdof = c.f(c.L.cdof);
  float* cvel = c.f(c.L.cvel);
  float* cdd = c.f(c.L.cdof_dot);
  float* cinert = c.f(c.L.cinert);
  float* qs = c.f(c.L.qfrc_smooth);
  // Actuator tables (lane = actuator, nu <= 64), with the transmission's dof or first
  // two tendon wraps, loaded now so that their L2 round trips (two of them dependent)
  // overlap the tree sums instead of following the barriers below.
  const int ia = min(LANE, max(c.nu - 1, 0));
  const bool a_ok = LANE < c.nu;
  const int a_trn = a_ok ? m.actuator_trntype[ia] : 0, a_id = a_ok ? m.actuator_trnid[ia] : 0;
  const int a_clim = a_ok ? m.actuator_ctrllimited[ia] : 0, a_flim = a_ok ? m.actuator_forcelimited[ia] : 0;
  const int a_bt = a_ok ? m.actuator_biastype[ia] : 0;
  const float a_g = a_ok ? m.actuator_gear[ia] : 0.f, a_gain = a_ok ? m.actuator_gainprm[3 * ia] : 0.f;
  const float a_c0 = a_ok ? m.actuator_ctrlrange[2 * ia] : 0.f, a_c1 = a_ok ? m.actuator_ctrlrange[2 * ia + 1] : 0.f;
  const float a_f0 = a_ok ? m.actuator_forcerange[2 * ia] : 0.f, a_f1 = a_ok ? m.actuator_forcerange[2 * ia + 1] : 0.f;
  const float a_b0 = a_ok ? m.actuator_biasprm[3 * ia] : 0.f, a_b1 = a_ok ? m.actuator_biasprm[3 * ia + 1] : 0.f,
              a_b2 = a_ok ? m.actuator_biasprm[3 * ia + 2] : 0.f;
  const int a_dof = (a_ok && a_trn == 0) ? m.jnt_dofadr[a_id] : 0;
  const int a_wa = (a_ok && a_trn != 0) ? m.tendon_adr[a_id] : 0;
  const int a_wn = (a_ok && a_trn != 0) ? m.tendon_num[a_id] : 0;
  const float a_wc0 = a_wn > 0 ? m.wrap_coef[a_wa] : 0.f, a_wc1 = a_wn > 1 ? m.wrap_coef[a_wa + 1] : 0.f;
  const int a_wd0 = a_wn > 0 ? m.wrap_dof[a_wa] : 0, a_wd1 = a_wn > 1 ? m.wrap_dof[a_wa + 1] : 0;
  // The tree recursions of mj_comVel / mj_rne are sums over a body's dof chain (the
  // dofs on its path to the root, dx_api.hip body_chain), so every dof and every body
  // is computed at once instead of one tree level after another:
  //   cdof_dot[d] = (sum of cdof[e] qvel[e] over the chain dofs e before d) x cdof[d]
  //   cvel[b]     = sum over chain(b) of cdof[e] qvel[e]
  //   cacc[b]     = -gravity + sum over chain(b) of cdof_dot[e] qvel[e]
  //   qfrc_bias[d] = cdof[d] . (sum of cfrc over the subtree of d's body)
  //               = sum over the bodies b whose chain holds d of cdof[d] . cfrc[b]
  // A free joint's rotational dofs see the velocity after its translation only, and
  // its translational cdof_dot is zero (mj_comVel).
  for (int d = LANE; d < nv; d += DX_WAVE) {  // lane = dof
    const float4 d0 = m.dof_rec[2 * d], d1 = m.dof_rec[2 * d + 1];
    const int tk = __float_as_int(d0.w), k = tk >> 8;
    const bool fr = (tk & 255) == DXJ_FREE;
    const uint64_t anc = (uint64_t)(uint32_t)__float_as_int(d1.z) | ((uint64_t)(uint32_t)__float_as_int(d1.w) << 32);
    uint64_t mask = anc & ((1ull << (fr ? d - k + 3 : d)) - 1ull);  // d - k + 3 <= d + 3 <= 63 (nv <= 64 model check)
    float cv[6] = {0, 0, 0, 0, 0, 0};
    while (mask) {
      const int e = __ffsll((long long)mask) - 1;
      mask &= mask - 1;
      const float q = qvel[e];
#pragma unroll
      for (int x = 0; x < 6; x++) cv[x] += cdof[6 * e + x] * q;
    }
    float o[6];
    cross_motion(o, cv, cdof + 6 * d);
#pragma unroll
    for (int x = 0; x < 6; x++) cdd[6 * d + x] = fr && k < 3 ? 0.f : o[x];
    qs[d] = -d1.y * qvel[d];  // passive damping; bias and actuation are added below
  }
  if (LANE < 6) cvel[LANE] = 0;
  SYNC();
  {  // lane = body
    const int b = LANE;
    const bool act = b >= 1 && b < c.nbody;
    const uint64_t ch = act ? m.body_chain[b] : 0ull;
    float cv[6] = {0, 0, 0, 0, 0, 0};
    float ca[6] = {0, 0, 0, -m.gravity[0], -m.gravity[1], -m.gravity[2]};
    for (uint64_t mask = ch; mask; mask &= mask - 1) {
      const int e = __ffsll((long long)mask) - 1;
      const float q = qvel[e];
#pragma unroll
      for (int x = 0; x < 6; x++) {
        cv[x] += cdof[6 * e + x] * q;
        ca[x] += cdd[6 * e + x] * q;
      }
    }
    if (act) {
#pragma unroll
      for (int x = 0; x < 6; x++) cvel[6 * b + x] = cv[x];
      // body force: I a + v x* I v - applied wrench (as com-frame spatial force)
      float t1[6], t2[6], t3[6], f[6];
      mul_inert(t1, cinert + 10 * b, ca);
      mul_inert(t2, cinert + 10 * b, cv);
      cross_force(t3, cv, t2);
#pragma unroll
      for (int x = 0; x < 6; x++) f[x] = t1[x] + t3[x];
      if (xfrc) {
        float f6[6];
        for (int x = 0; x < 6; x++) f6[x] = xfrc[6 * b + x];
        if (f6[0] != 0 || f6[1] != 0 || f6[2] != 0 || f6[3] != 0 || f6[4] != 0 || f6[5] != 0) {
          const int rootidx = __float_as_int(m.body_rec[8 * b + 3].w);
          const float* rc = c.f(c.L.rcom) + 3 * rootidx;
          const float* xi = c.f(c.L.xipos) + 3 * b;
          float off[3] = {xi[0] - rc[0], xi[1] - rc[1], xi[2] - rc[2]};
          float tq[3];
          cross3(tq, off, f6);
          f[0] -= f6[3] + tq[0];
          f[1] -= f6[4] + tq[1];
          f[2] -= f6[5] + tq[2];
          f[3] -= f6[0];
          f[4] -= f6[1];
          f[5] -= f6[2];
        }
      }
      // qfrc_smooth = passive - (bias - applied) + actuator: this body's share of
      // the bias of every dof on its chain
      for (uint64_t mask = ch; mask; mask &= mask - 1) {
        const int e = __ffsll((long long)mask) - 1;
        atomicAdd(qs + e, -dot6(cdof + 6 * e, f));
      }
    }
  }
  SYNC();
  float* al = c.f(c.L.act_len);
  float* ctrl = c.f(c.L.ctrl);
  float* tl = c.f(c.L.ten_len);
  (void)tl;
  if (a_ok) {
    const int i = LANE;
    float cc = ctrl[i];
    if (a_clim) cc = fminf(a_c1, fmaxf(a_c0, cc));
    const float g = a_g;
    float vel;
    if (a_trn == 0) {
      vel = g * qvel[a_dof];
    } else {
      vel = 0;
      for (int w = 0; w < a_wn; w++) {
        const float wc = w == 0 ? a_wc0 : (w == 1 ? a_wc1 : m.wrap_coef[a_wa + w]);
        const int wd = w == 0 ? a_wd0 : (w == 1 ? a_wd1 : m.wrap_dof[a_wa + w]);
        vel += g * wc * qvel[wd];
      }
    }
    float force = a_gain * cc;
    if (a_bt == 1) force += a_b0 + a_b1 * al[i] + a_b2 * vel;
    if (a_flim) force = fminf(a_f1, fmaxf(a_f0, force));
    if (a_trn == 0) {
      atomicAdd(qs + a_dof, g * force);
    } else {
      for (int w = 0; w < a_wn; w++) {
        const float wc = w == 0 ? a_wc0 : (w == 1 ? a_wc1 : m.wrap_coef[a_wa + w]);
        const int wd = w == 0 ? a_wd0 : (w == 1 ? a_wd1 : m.wrap_dof[a_wa + w]);
        atomicAdd(qs + wd, g * wc * force);
      }
    }
  }
  SYNC();
}

// ------------------------------------------------------------------------ //
// Newton solver
// ------------------------------------------------------------------------ //
// The force and Hessian weight of row_cost by selects (the line searches' inner loops:
// the lanes hold rows of every type and zone at once, so row_cost's early returns were
// exec-mask branches taken both ways).  The same zones and values.
__device__ __forceinline__ void row_force(int type, float D, float fl, float Rf, float jar, float& force, float& hw) {
  const bool fr = type == DXR_FRIC;
  const bool lo = fr && jar <= -Rf, hi = fr && jar >= Rf;  // friction's linear zones
  const bool quad = fr ? !(lo || hi) : jar < 0;             // the quadratic zone
  force = lo ? fl : hi ? -fl : quad ? -D * jar : 0.f;
  hw = quad ? D : 0.f;
}
// row cost at jar -> (cost, force, hessian weight)
__device__ __forceinline__ float row_cost(int type, float D, float fl, float Rf, float jar, float& force, float& hw) {
  row_force(type, D, fl, Rf, jar, force, hw);
  const bool fr = type == DXR_FRIC;
  const bool lo = fr && jar <= -Rf, hi = fr && jar >= Rf;
  const bool quad = fr ? !(lo || hi) : jar < 0;
  return lo ? -fl * jar - 0.5f * Rf * fl : hi ? fl * jar - 0.5f * Rf * fl : quad ? 0.5f * D * jar * jar : 0.f;
}

// y = M x (lanes over rows).  For n <= 32 the row is gathered with 32 independent
// LDS reads (one latency, not one per element).  Columns past n read a clamped,
// in-range address and are zeroed after the load: a guarded load would be a branch
// with its own LDS wait per column.
__device__ __forceinline__ void mat_vec(const float* M, const float* x, float* y, int n) {
  const int i = min(LANE, n - 1);
  if (n <= 32) {
    float s = 0;
#pragma unroll
    for (int k = 0; k < 32; k++) {
      const int kc = min(k, n - 1);
      const float xv = x[kc], mv = M[ti(max(i, kc)) + min(i, kc)];
      s = fmaf(k < n ? mv : 0.f, xv, s);
    }
    if (LANE < n) y[LANE] = s;
    return;
  }
  // n <= 64 (DX_MAX_NV): the same unrolled gather over 64 columns, every read
  // independent of the running sum
  float s = 0;
#pragma unroll
  for (int k = 0; k < 64; k++) {
    const int kc = min(k, n - 1);
    const float xv = x[kc], mv = M[ti(max(i, kc)) + min(i, kc)];
    s = fmaf(k < n ? mv : 0.f, xv, s);
  }
  if (LANE < n) y[LANE] = s;
}

// n <= 30: lane i holds row i of the packed symmetric M in registers (0 past n), loaded
// once per solve; M x is then 30 readlanes of x and 30 FMAs per lane -- no LDS gather and
// no packed-index arithmetic per product (the Newton solve takes ~4.4 per substep).
__device__ __forceinline__ void mrow_load(const float* M, int n, float (&mr)[30]) {
  const int i = min(LANE, n - 1);
#pragma unroll
  for (int k = 0; k < 30; k++) {
    const int kc = min(k, n - 1);
    const float t = M[ti(max(i, kc)) + min(i, kc)];
    mr[k] = LANE < n && k < n ? t : 0.f;
  }
}
__device__ __forceinline__ void mat_vec_rows(const float (&mr)[30], const float* x, float* y, int n) {
  const float xi = x[min(LANE, n - 1)];
  float s0 = 0.f, s1 = 0.f;
#pragma unroll
  for (int k = 0; k < 30; k += 2) {
    s0 = fmaf(mr[k], rl(xi, k), s0);
    s1 = fmaf(mr[k + 1], rl(xi, k + 1), s1);
  }
  if (LANE < n) y[LANE] = s0 + s1;
}
__device__ float dx_mrow_none[30];  // (the reference line_search / eval_cost take when MREG is off)

template <class Ctx>
__device__ __forceinline__ void jac_rows(const Ctx& c, const float* x, float* out);
// J x for every row -> out[r]; uses cq as contact-frame scratch.  The contact
// frame rows are gathered with DX_DOFMAX independent reads per lane.
template <class Ctx>
__device__ __forceinline__ void jac_vec(const Ctx& c, const float* x, float* out) {
  int ncon = c.I[I_NCON];
  const unsigned char* cj_idx = (const unsigned char*)c.f(c.L.cj_idx);
  const float* cj_val = c.f(c.L.cj_val);
  float* cq = c.f(c.L.cq);
  const float* con = c.f(c.L.con);
  for (int t = LANE; t < 3 * ncon; t += DX_WAVE) {
    int ci = t / 3, k = t - 3 * ci;
    int nnz = __float_as_int(con[DX_CON_STRIDE * ci + 14]) & 255;
    float s = 0;
#pragma unroll
    for (int q = 0; q < DX_DOFMAX; q++) {  // unguarded loads; slots past nnz are not summed
      const float v = cj_val[(ci * 3 + k) * DX_DOFMAX + q];
      const float xv = x[cj_idx[ci * DX_DOFMAX + q]];
      const float t = fmaf(v, xv, s);
      s = q < nnz ? t : s;
    }
    cq[t] = s;
  }
  SYNC();
  jac_rows(c, x, out);
}
// the rows of J x from the contact-frame products in cq (jac_vec's second pass)
template <class Ctx>
__device__ __forceinline__ void jac_rows(const Ctx& c, const float* x, float* out) {
  const DevModel& m = c.mdl();
  const int nefc = c.I[I_NEFC];
  const int* meta = (const int*)c.f(c.L.efc_meta);
  const float* cq = c.f(c.L.cq);
  const float* con = c.f(c.L.con);
  for (int r = LANE; r < nefc; r += DX_WAVE) {
    int mt = meta[r], type = mt & 15, aux = (mt >> 4) & 15, id = mt >> 8;
    float v;
    if (type == DXR_FRIC) v = x[id];
    else if (type == DXR_LIMJ) v = aux == 0 ? x[id] : -x[id];
    else if (type == DXR_LIMT) {
      v = 0;
      for (int w = m.tendon_adr[id]; w < m.tendon_adr[id] + m.tendon_num[id]; w++) v += m.wrap_coef[w] * x[m.wrap_dof[w]];
      if (aux) v = -v;
    } else if (type == DXR_CONFL) {
      v = cq[3 * id];
    } else {
      int k = 1 + (aux >> 1);
      float mu = con[DX_CON_STRIDE * id + 15 + k] * ((aux & 1) ? -1.f : 1.f);
      v = cq[3 * id] + mu * cq[3 * id + k];
    }
    out[r] = v;
  }
  SYNC();
}

// sum of the constraint rows' costs at residuals jr (+ g0, the Gauss term)
template <class Ctx>
__device__ __forceinline__ float rows_cost(const Ctx& c, const float* jr, float g0) {
  const DevModel& m = c.mdl();
  int nefc = c.I[I_NEFC];
  const int* meta = (const int*)c.f(c.L.efc_meta);
  const float* D = c.f(c.L.efc_D);
  const float* fl = c.f(c.L.efc_fl);
  const float* Rf = c.f(c.L.efc_Rf);
  float g = g0;
  for (int r = LANE; r < nefc; r += DX_WAVE) {
    float f, hw;
    bool fr = r < c.nfric;
    g += row_cost(meta[r] & 15, D[r], fr ? fl[r] : 0.f, fr ? Rf[r] : 0.f, jr[r], f, hw);
  }
  (void)m;
  return wave_sum(g);
}

// cost at the current jar (efc_jar) + gauss; fills nothing else.  Returns total.
template <class Ctx>
__device__ __forceinline__ float total_cost(const Ctx& c, const float* qacc, const float* Ma, float* gauss = nullptr) {
  const DevModel& m = c.mdl();
  int nv = c.nv;
  const float* qs = c.f(c.L.qfrc_smooth);
  const float* a0 = c.f(c.L.qacc_smooth);
  float g = 0;
  for (int i = LANE; i < nv; i += DX_WAVE) g += 0.5f * (qacc[i] - a0[i]) * (Ma[i] - qs[i]);
  if (gauss) *gauss = wave_sum(g);
  int nefc = c.I[I_NEFC];
  const int* meta = (const int*)c.f(c.L.efc_meta);
  const float* D = c.f(c.L.efc_D);
  const float* fl = c.f(c.L.efc_fl);
  const float* Rf = c.f(c.L.efc_Rf);
  const float* jar = c.f(c.L.efc_jar);
  for (int r = LANE; r < nefc; r += DX_WAVE) {
    float f, hw;
    bool fr = r < c.nfric;
    g += row_cost(meta[r] & 15, D[r], fr ? fl[r] : 0.f, fr ? Rf[r] : 0.f, jar[r], f, hw);
  }
  return wave_sum(g);
}

// jar = J qacc - aref, Ma = M qacc; returns cost
template <bool MREG = false, class Ctx>
__device__ __forceinline__ float eval_cost(const Ctx& c, const float* qacc, float* Ma, float* gauss = nullptr,
                                           const float (&mr)[30] = dx_mrow_none) {
  int nv = c.nv;
  if (MREG) mat_vec_rows(mr, qacc, Ma, nv);
  else mat_vec(c.f(c.L.M), qacc, Ma, nv);
  stage_mark(c, ST_MATVEC);
  float* jar = c.f(c.L.efc_jar);
  jac_vec(c, qacc, jar);
  stage_mark(c, ST_JACVEC);
  const float* aref = c.f(c.L.efc_aref);
  int nefc = c.I[I_NEFC];
  for (int r = LANE; r < nefc; r += DX_WAVE) jar[r] -= aref[r];
  SYNC();
  return total_cost(c, qacc, Ma, gauss);
}

// out[d] = sum_r J[r][d] * w[r] computed as J^T applied to the per-row force of the
// current jar (force mode) -- lane per dof, deterministic.
template <class Ctx>
__device__ __forceinline__ void jac_t_force(const Ctx& c, float* out) {
  const DevModel& m = c.mdl();
  int nv = c.nv;
  int nefc = c.I[I_NEFC];
  int ncon = c.I[I_NCON];
  const int* meta = (const int*)c.f(c.L.efc_meta);
  const float* D = c.f(c.L.efc_D);
  const float* fl = c.f(c.L.efc_fl);
  const float* Rf = c.f(c.L.efc_Rf);
  const float* jar = c.f(c.L.efc_jar);
  const float* con = c.f(c.L.con);
  float* cw = c.f(c.L.cw);  // contact frame forces [ncon][3]
  // contact frame forces
  for (int ci = LANE; ci < ncon; ci += DX_WAVE) {
    const float* r = con + DX_CON_STRIDE * ci;
    int row0 = __float_as_int(r[15]);
    float fc[3] = {0, 0, 0};
    if ((__float_as_int(r[14]) >> 8) == 1) {
      float f, hw;
      if (row0 < nefc) { row_force(DXR_CONFL, D[row0], 0, 0, jar[row0], f, hw); fc[0] = f; }
    } else {
      for (int e = 0; e < 4; e++) {
        int row = row0 + e;
        if (row >= nefc) break;
        float f, hw;
        row_force(DXR_CON, D[row], 0, 0, jar[row], f, hw);
        int k = 1 + (e >> 1);
        float mu = r[15 + k] * ((e & 1) ? -1.f : 1.f);
        fc[0] += f;
        fc[k] += mu * f;
      }
    }
    cw[3 * ci] = fc[0]; cw[3 * ci + 1] = fc[1]; cw[3 * ci + 2] = fc[2];
  }
  SYNC();
  const unsigned char* cj_idx = (const unsigned char*)c.f(c.L.cj_idx);
  const float* cj_val = c.f(c.L.cj_val);
  for (int d = LANE; d < nv; d += DX_WAVE) {
    float s = 0;
    // friction row of this dof
    int fr = m.dof_fricrow[d];
    if (fr >= 0) { float f, hw; row_force(DXR_FRIC, D[fr], fl[fr], Rf[fr], jar[fr], f, hw); s += f; }
    for (int r = c.nfric; r < nefc; r++) {
      int mt = meta[r], type = mt & 15, aux = (mt >> 4) & 15, id = mt >> 8;
      if (type == DXR_LIMJ) {
        if (id != d) continue;
        float f, hw;
        row_force(type, D[r], 0, 0, jar[r], f, hw);
        s += aux ? -f : f;
      } else if (type == DXR_LIMT) {
        float tj = m.tendon_J[id * nv + d];
        if (tj == 0) continue;
        float f, hw;
        row_force(type, D[r], 0, 0, jar[r], f, hw);
        s += (aux ? -tj : tj) * f;
      } else {
        break;  // contact rows are last
      }
    }
    out[d] = s;
  }
  SYNC();
  // the contacts, over (contact, support slot) items (16 slots a contact): lane (ci, q)
  // adds its slot's J^T f term to its dof with an LDS float atomic.  Within one atomic
  // the lanes of a dof are applied in lane order, i.e. contact order, as the serial sum
  // of each dof's contacts did (one lane per dof, a loop over the contacts: ncon
  // dependent rounds of LDS reads, the bulk of the solvers' gradient stage).
  const int nitem = 16 * ncon;
  for (int base = 0; base < nitem; base += DX_WAVE) {
    const int t = base + LANE;
    const int ci = min(t >> 4, max(ncon - 1, 0)), q = t & 15;
    const int nnz = __float_as_int(con[DX_CON_STRIDE * ci + 14]) & 255;
    if (t < nitem && q < nnz) {
      const int d = cj_idx[ci * DX_DOFMAX + q];
      const float* cv = cj_val + ci * 3 * DX_DOFMAX + q;
      const float tv = cv[0] * cw[3 * ci] + cv[DX_DOFMAX] * cw[3 * ci + 1] + cv[2 * DX_DOFMAX] * cw[3 * ci + 2];
      atomicAdd(out + d, tv);
    }
  }
  SYNC();
}

// H = M + J^T D_active J  (at the current jar)
template <class Ctx>
__device__ __forceinline__ void build_hessian(const Ctx& c) {
  const DevModel& m = c.mdl();
  int nv = c.nv;
  int nefc = c.I[I_NEFC];
  int ncon = c.I[I_NCON];
  float* H = c.f(c.L.H);
  const float* M = c.f(c.L.M);
  const int* meta = (const int*)c.f(c.L.efc_meta);
  const float* D = c.f(c.L.efc_D);
  const float* fl = c.f(c.L.efc_fl);
  const float* Rf = c.f(c.L.efc_Rf);
  const float* jar = c.f(c.L.efc_jar);
  for (int k = LANE; k < ti(nv); k += DX_WAVE) H[k] = M[k];
  SYNC();
  // unit rows (friction, joint limits) -> diagonal; lane per dof
  for (int d = LANE; d < nv; d += DX_WAVE) {
    float s = 0;
    int fr = m.dof_fricrow[d];
    if (fr >= 0) { float f, hw; row_force(DXR_FRIC, D[fr], fl[fr], Rf[fr], jar[fr], f, hw); s += hw; }
    for (int r = c.nfric; r < nefc; r++) {
      int mt = meta[r], type = mt & 15, id = mt >> 8;
      if (type != DXR_LIMJ) { if (type == DXR_LIMT) continue; break; }
      if (id != d) continue;
      float f, hw;
      row_force(type, D[r], 0, 0, jar[r], f, hw);
      s += hw;
    }
    H[ti(d) + d] += s;
  }
  SYNC();
  // tendon limit rows: dense outer products, lanes over entries
  for (int r = c.nfric; r < nefc; r++) {
    int mt = meta[r], type = mt & 15, id = mt >> 8;
    if (type == DXR_CON || type == DXR_CONFL) break;
    if (type != DXR_LIMT) continue;
    float f, hw;
    row_force(type, D[r], 0, 0, jar[r], f, hw);
    if (hw == 0) continue;
    const float* tj = m.tendon_J + id * nv;
    for (int i = LANE; i < nv; i += DX_WAVE)
      for (int j = 0; j <= i; j++) H[ti(i) + j] += hw * tj[i] * tj[j];
    SYNC();
  }
  // contacts: W = sum_active_edges D c c^T in frame space; H[idx_a][idx_b] += J^T W J.
  // Lane ci < ncon builds contact ci's W (symmetric: w00, w01, w02, w11, w22); then
  // the lower-triangle items of every contact's nnz x nnz block are flattened over
  // the lanes (item t -> contact by a 5-step search over the lanes' prefix counts)
  // and summed into H with LDS float atomics, so contacts no longer run one after
  // another (a contact-rich env has ~20 of them).
  const float* con = c.f(c.L.con);
  const unsigned char* cj_idx = (const unsigned char*)c.f(c.L.cj_idx);
  const float* cj_val = c.f(c.L.cj_val);
#pragma unroll 1
  for (int ch = 0; ch < DX_NCH; ch++) {  // contact chunks (lane = contact)
    const int cb = ch * DX_WAVE;
    if (cb >= ncon) break;  // uniform
    const int nc = min(ncon - cb, DX_WAVE);
    float w00 = 0.f, w01 = 0.f, w02 = 0.f, w11 = 0.f, w22 = 0.f;
    int nnz = 0, items = 0;
    if (LANE < nc) {
      const float* r = con + DX_CON_STRIDE * (cb + LANE);
      const int row0 = __float_as_int(r[15]);
      nnz = __float_as_int(r[14]) & 255;
      if ((__float_as_int(r[14]) >> 8) == 1) {
        if (row0 < nefc) {
          float f, hw;
          row_force(DXR_CONFL, D[row0], 0, 0, jar[row0], f, hw);
          w00 = hw;
        }
      } else {
        for (int e = 0; e < 4; e++) {
          const int row = row0 + e;
          if (row >= nefc) break;
          float f, hw;
          row_force(DXR_CON, D[row], 0, 0, jar[row], f, hw);
          const float mu = r[16 + (e >> 1)] * ((e & 1) ? -1.f : 1.f);
          w00 += hw;
          if (e < 2) { w01 += hw * mu; w11 += hw * mu * mu; }
          else { w02 += hw * mu; w22 += hw * mu * mu; }
        }
      }
      items = (w00 == 0.f && w11 == 0.f && w22 == 0.f) ? 0 : nnz * (nnz + 1) / 2;
    }
    const int incl = wave_incl_scan(items);
    const int excl = incl - items;
    const int total = __builtin_amdgcn_readlane(incl, 63);
    for (int base = 0; base < total; base += DX_WAVE) {  // uniform trip count: the shuffles see every lane
      const int t = min(base + LANE, total - 1);
      int ci = 0;  // last contact whose first item is <= t (contacts without items tie and lose)
#pragma unroll
      for (int st = DX_SEARCH0; st >= 1; st >>= 1) {
        const int mid = ci + st;
        const int em = __shfl(excl, mid & 63, 64);
        if (mid < nc && em <= t) ci = mid;
      }
      const int u = t - __shfl(excl, ci, 64);
      int a = (int)((sqrtf(8.0f * (float)u + 1.0f) - 1.0f) * 0.5f);
      a += (a + 1) * (a + 2) / 2 <= u;
      a -= a * (a + 1) / 2 > u;
      const int b = u - a * (a + 1) / 2;
      const float c00 = __shfl(w00, ci, 64), c01 = __shfl(w01, ci, 64), c02 = __shfl(w02, ci, 64);
      const float c11 = __shfl(w11, ci, 64), c22 = __shfl(w22, ci, 64);
      const int cg = cb + ci;
      const float* jv = cj_val + cg * 3 * DX_DOFMAX;
      const float a0 = jv[a], a1 = jv[DX_DOFMAX + a], a2 = jv[2 * DX_DOFMAX + a];
      const float b0 = jv[b], b1 = jv[DX_DOFMAX + b], b2 = jv[2 * DX_DOFMAX + b];
      const float sum = c00 * a0 * b0 + c01 * (a0 * b1 + a1 * b0) + c02 * (a0 * b2 + a2 * b0) + c11 * a1 * b1 +
                        c22 * a2 * b2;
      if (base + LANE < total) atomicAdd(H + ti(cj_idx[cg * DX_DOFMAX + a]) + cj_idx[cg * DX_DOFMAX + b], sum);
    }
  }
  SYNC();
}

// Incremental Hessian for the sweep solve (nv <= 30, no tendon-limit rows).  H in LDS
// holds M + sum_contacts J_c^T W_c J_c and is not touched by the sweep, so after the
// first build only the contacts whose W changed in the last line search add their
// change, (W_new - W_old) -- MuJoCo's Newton likewise updates its factor only for the
// constraints whose state changed ([3P] mj_solNewton's incremental Hessian).  Lane ci
// keeps contact ci's W (wo) across iterations.  The unit rows' diagonal (friction loss,
// joint limits) is rebuilt every iteration into a register, the sweep's diagonal
// addition for column LANE % 32.  Returns that addition.
template <class Ctx>
__device__ __forceinline__ float build_hessian_inc(const Ctx& c, bool first, float (&wo)[DX_NCH][5]) {
  const DevModel& m = c.mdl();
  const int nv = c.nv;
  const int nefc = c.I[I_NEFC];
  const int ncon = c.I[I_NCON];
  float* H = c.f(c.L.H);
  const int* meta = (const int*)c.f(c.L.efc_meta);
  const float* D = c.f(c.L.efc_D);
  const float* fl = c.f(c.L.efc_fl);
  const float* Rf = c.f(c.L.efc_Rf);
  const float* jar = c.f(c.L.efc_jar);
  if (first) {
    const float* M = c.f(c.L.M);
    for (int k = LANE; k < ti(nv); k += DX_WAVE) H[k] = M[k];
  }
  // unit rows (friction, joint limits) -> this lane's diagonal addition
  float s = 0.f;
  {
    const int d = LANE & 31;
    if (d < nv) {
      const int fr = m.dof_fricrow[d];
      if (fr >= 0) { float f, hw; row_force(DXR_FRIC, D[fr], fl[fr], Rf[fr], jar[fr], f, hw); s += hw; }
      for (int r = c.nfric; r < nefc; r++) {
        const int mt = meta[r], type = mt & 15, id = mt >> 8;
        if (type != DXR_LIMJ) break;  // (no tendon-limit rows on this path)
        if (id != d) continue;
        float f, hw;
        row_force(type, D[r], 0, 0, jar[r], f, hw);
        s += hw;
      }
    }
  }
  const float* con = c.f(c.L.con);
  const unsigned char* cj_idx = (const unsigned char*)c.f(c.L.cj_idx);
  const float* cj_val = c.f(c.L.cj_val);
  constexpr int NCH = DX_NCH;  // contact chunks (lane = contact)
#pragma unroll
  for (int ch = 0; ch < NCH; ch++) {
    const int cb = ch * DX_WAVE;
    if (cb >= ncon) break;  // uniform
    const int nc = min(ncon - cb, DX_WAVE);
    float w[5] = {0.f, 0.f, 0.f, 0.f, 0.f};  // w00, w01, w02, w11, w22
    int nnz = 0;
    if (LANE < nc) {
      const float* r = con + DX_CON_STRIDE * (cb + LANE);
      const int row0 = __float_as_int(r[15]);
      nnz = __float_as_int(r[14]) & 255;
      if ((__float_as_int(r[14]) >> 8) == 1) {
        if (row0 < nefc) {
          float f, hw;
          row_force(DXR_CONFL, D[row0], 0, 0, jar[row0], f, hw);
          w[0] = hw;
        }
      } else {
        for (int e = 0; e < 4; e++) {
          const int row = row0 + e;
          if (row >= nefc) break;
          float f, hw;
          row_force(DXR_CON, D[row], 0, 0, jar[row], f, hw);
          const float mu = r[16 + (e >> 1)] * ((e & 1) ? -1.f : 1.f);
          w[0] += hw;
          if (e < 2) { w[1] += hw * mu; w[3] += hw * mu * mu; }
          else { w[2] += hw * mu; w[4] += hw * mu * mu; }
        }
      }
    }
    float dw[5];
    bool chg = false;
#pragma unroll
    for (int k = 0; k < 5; k++) {
      dw[k] = w[k] - wo[ch][k];
      chg |= w[k] != wo[ch][k];
      wo[ch][k] = w[k];
    }
    const int items = chg ? nnz * (nnz + 1) / 2 : 0;
    const int incl = wave_incl_scan(items);
    const int excl = incl - items;
    const int total = __builtin_amdgcn_readlane(incl, 63);
    if (first && ch == 0) SYNC();  // the M copy before the atomics
    for (int base = 0; base < total; base += DX_WAVE) {  // uniform trip count: the shuffles see every lane
      const int t = min(base + LANE, total - 1);
      int ci = 0;  // last contact whose first item is <= t (contacts without items tie and lose)
#pragma unroll
      for (int st = DX_SEARCH0; st >= 1; st >>= 1) {
        const int mid = ci + st;
        const int em = __shfl(excl, mid & 63, 64);
        if (mid < nc && em <= t) ci = mid;
      }
      const int u = t - __shfl(excl, ci, 64);
      int a = (int)((sqrtf(8.0f * (float)u + 1.0f) - 1.0f) * 0.5f);
      a += (a + 1) * (a + 2) / 2 <= u;
      a -= a * (a + 1) / 2 > u;
      const int b = u - a * (a + 1) / 2;
      const float c00 = __shfl(dw[0], ci, 64), c01 = __shfl(dw[1], ci, 64), c02 = __shfl(dw[2], ci, 64);
      const float c11 = __shfl(dw[3], ci, 64), c22 = __shfl(dw[4], ci, 64);
      const int cg = cb + ci;
      const float* jv = cj_val + cg * 3 * DX_DOFMAX;
      const float a0 = jv[a], a1 = jv[DX_DOFMAX + a], a2 = jv[2 * DX_DOFMAX + a];
      const float b0 = jv[b], b1 = jv[DX_DOFMAX + b], b2 = jv[2 * DX_DOFMAX + b];
      const float sum = c00 * a0 * b0 + c01 * (a0 * b1 + a1 * b0) + c02 * (a0 * b2 + a2 * b0) + c11 * a1 * b1 +
                        c22 * a2 * b2;
      if (base + LANE < total) atomicAdd(H + ti(cj_idx[cg * DX_DOFMAX + a]) + cj_idx[cg * DX_DOFMAX + b], sum);
    }
  }
  SYNC();
  return s;
}

// zone of a row's cost at jar: 0 zero, 1 quadratic, 2 / 3 linear friction zones
__device__ __forceinline__ int row_zone(int type, float Rf, float jar) {
  if (type == DXR_FRIC) return jar <= -Rf ? 3 : (jar >= Rf ? 2 : 1);
  return jar < 0 ? 1 : 0;
}

// Exact line search along dir (1-D Newton with bracketing on the piecewise-quadratic
// cost).  Every row's (type, D, friction, jar, J dir) is loaded into registers once
// -- lane-owned rows r = LANE + 64 k -- so the iterations touch no LDS.
#ifndef DX_LS_SLOTS
#define DX_LS_SLOTS (DX_NCON_MAX > 64 ? 20 : 5)  // nefc_max <= 320 / 1280 (checked at model load)
#endif
// NEWTON (dir = -H^-1 grad): the slope at alpha = 0 is grad . dir and the curvature there
// dir^T H dir = -grad . dir (H is the Hessian of the zone set at alpha = 0), so the first
// 1-D Newton step from 0 lands at alpha = 1 -- the search starts there, with g0 = grad . dir
// -- and at the end the new residuals are written from the registers and the cost at the
// new point is returned in *cost_new: the rows' costs plus the Gauss term, continued along
// the line as gauss + alpha qb + alpha^2 qa / 2 (M qacc_smooth = qfrc_smooth), so the
// solver needs no separate cost pass.
// HAVE_MDIR: the caller already holds M dir in v4 (CG's recurrence), no product here.
// MREG: M's rows in registers (mrow_load), the product without LDS.
template <bool NEWTON = false, bool HAVE_MDIR = false, bool MREG = false, bool HAVE_JV = false, class Ctx>
__device__ __forceinline__ float line_search(const Ctx& c, const float* qacc, const float* Ma, const float* dir, int* changed,
                                             float* slope0 = nullptr, const float* grad = nullptr,
                                             float gauss = 0.f, float* cost_new = nullptr, float* gauss_new = nullptr,
                                             const float (&mr)[30] = dx_mrow_none) {
  const DevModel& m = c.mdl();
  int nv = c.nv;
  float* Mdir = c.f(c.L.v4);
  if (!HAVE_MDIR) {
    if (MREG) mat_vec_rows(mr, dir, Mdir, nv);
    else mat_vec(c.f(c.L.M), dir, Mdir, nv);
    stage_mark(c, ST_MATVEC);
  }
  float* jv = c.f(c.L.efc_jv);
  if (!HAVE_JV) {  // (HAVE_JV: the caller has J dir in efc_jv)
    jac_vec(c, dir, jv);  // includes SYNC
    stage_mark(c, ST_JACVEC);
  }
  const float* qs = c.f(c.L.qfrc_smooth);
  float qa = 0, qb = 0, qg = 0;
  for (int i = LANE; i < nv; i += DX_WAVE) {
    qa += dir[i] * Mdir[i];
    qb += dir[i] * (Ma[i] - qs[i]);
    if (NEWTON) qg += dir[i] * grad[i];
  }
  qa = wave_sum(qa);
  qb = wave_sum(qb);
  if (NEWTON) qg = wave_sum(qg);
  int nefc = c.I[I_NEFC];
  const int ns = (nefc + DX_WAVE - 1) / DX_WAVE;  // uniform
  const int* meta = (const int*)c.f(c.L.efc_meta);
  const float* Dp = c.f(c.L.efc_D);
  const float* flp = c.f(c.L.efc_fl);
  const float* Rfp = c.f(c.L.efc_Rf);
  const float* jarp = c.f(c.L.efc_jar);
  int ty[DX_LS_SLOTS];
  float D[DX_LS_SLOTS], fl[DX_LS_SLOTS], Rf[DX_LS_SLOTS], ja[DX_LS_SLOTS], jj[DX_LS_SLOTS];
#pragma unroll
  for (int k = 0; k < DX_LS_SLOTS; k++) {
    if (k < ns) {  // uniform; the loads read a clamped row and select after (no per-lane branch)
      const int r = LANE + DX_WAVE * k;
      const int rc = max(min(r, nefc - 1), 0);
      const bool ok = r < nefc;
      const bool fr = ok && r < c.nfric;
      const int mt = meta[rc];
      const float d = Dp[rc], f = flp[rc], rf = Rfp[rc], a = jarp[rc], v = jv[rc];
      ty[k] = ok ? (mt & 15) : DXR_CON;
      D[k] = ok ? d : 0.f;
      fl[k] = fr ? f : 0.f;
      Rf[k] = fr ? rf : 0.f;
      ja[k] = ok ? a : 0.f;
      jj[k] = ok ? v : 0.f;
    } else {
      ty[k] = DXR_CON;
      D[k] = fl[k] = Rf[k] = ja[k] = jj[k] = 0.f;
    }
  }
  float lo = 0, hi = -1, alpha = 0, g0 = 0;
  int it = 0;
  if (NEWTON) {
    g0 = qg;
    if (g0 < 0.f) { alpha = 1.f; it = 1; }  // else not a descent direction: alpha stays 0
    else it = 40;
  }
  for (; it < 40; it++) {
    float g = 0, h = 0;
#pragma unroll
    for (int k = 0; k < DX_LS_SLOTS; k++) {
      if (k < ns) {
        float f, hw;
        row_force(ty[k], D[k], fl[k], Rf[k], ja[k] + alpha * jj[k], f, hw);
        g -= f * jj[k];
        h += hw * jj[k] * jj[k];
      }
    }
    g = wave_sum(g) + qa * alpha + qb;
    h = wave_sum(h) + qa;
    if (it == 0) g0 = g;
    if (fabsf(g) <= 1e-6f * fabsf(g0)) break;
    if (g < 0) lo = alpha; else hi = alpha;
    float next = h > 0 ? alpha - g / h : alpha + 1;
    if (hi >= 0 && (next <= lo || next >= hi)) next = 0.5f * (lo + hi);
    if (hi < 0 && next <= lo) next = lo + 1;
    if (fabsf(next - alpha) <= 1e-7f * fabsf(alpha)) break;
    alpha = next;
  }
  stage_count(c, CNT_LS_IT, min(it + 1, 40));
  if (slope0) *slope0 = g0;
  if (NEWTON) {
    float* jw = c.f(c.L.efc_jar);
    float rc = 0.f;
#pragma unroll
    for (int k = 0; k < DX_LS_SLOTS; k++) {
      if (k < ns) {
        const float jn = ja[k] + alpha * jj[k];
        float f, hw;
        rc += row_cost(ty[k], D[k], fl[k], Rf[k], jn, f, hw);
        const int r = LANE + DX_WAVE * k;
        if (r < nefc) jw[r] = jn;
      }
    }
    const float gn = gauss + alpha * qb + 0.5f * alpha * alpha * qa;
    *gauss_new = gn;
    *cost_new = gn + wave_sum(rc);
  }
  // rows whose cost zone differs between the current point and the new one
  int ch = 0;
#pragma unroll
  for (int k = 0; k < DX_LS_SLOTS; k++)
    if (k < ns) ch += jj[k] != 0.f && row_zone(ty[k], Rf[k], ja[k]) != row_zone(ty[k], Rf[k], ja[k] + alpha * jj[k]);
  *changed = wave_sum_i(ch);
  return alpha;
}

// solve_cg for nv <= 30 and up to 128 rows, every vector in registers (round 6): lane d
// holds qacc, M qacc, qfrc_smooth, grad, M^-1 grad, dir and M dir of dof d, lanes r and
// 64 + r hold rows r / 64 + r -- J's row dense (30 registers), its type, D, floss, R and
// residual.  M^-1 grad and M x are 30 readlanes and FMAs against the matrices' rows in
// registers, J dir one FMA per dof in the row's lane, J'f a reduce-scatter of every lane's
// f_r J_r (wave_reduce_scatter32); the exact line search runs on the row registers.  No LDS
// vector, no contact-frame pass and no atomic per iteration: what is left on the chain is
// the wave sums of the dot products.  The same algorithm and tests as solve_cg.
template <class Ctx, class F>
__device__ __forceinline__ void pgs_row_nz(const Ctx& c, int k, F&& add);
template <class Ctx>
__device__ __forceinline__ void solve_cg_reg(const Ctx& c, float scale, float tol) {
  const int nv = c.nv, nefc = c.I[I_NEFC];
  const int lane = LANE;
  const bool dof = lane < nv;
  const int dc = min(lane, nv - 1);
  float* qacc = c.f(c.L.qacc);
  float* Ma = c.f(c.L.v1);
  float* jar = c.f(c.L.efc_jar);
  const float* M = c.f(c.L.M);
  const float* qs = c.f(c.L.qfrc_smooth);
  float* T = c.f(c.L.H);
  float x = dof ? qacc[dc] : 0.f, ma = dof ? Ma[dc] : 0.f, q0 = dof ? qs[dc] : 0.f;
  float trow[30], mrow[30];  // lane i: row i of M^-1 and of M
  mfma_sweep_inverse30(M, nv, T);
  mrow_load(T, nv, trow);
  mrow_load(M, nv, mrow);
  const int* meta = (const int*)c.f(c.L.efc_meta);
  const float* Dp = c.f(c.L.efc_D);
  const float* flp = c.f(c.L.efc_fl);
  const float* Rfp = c.f(c.L.efc_Rf);
  float Jd[2][30];
  int ty[2];
  float D[2], fl[2], Rf[2], ja[2], jj[2];
#pragma unroll
  for (int h = 0; h < 2; h++) {
    const int r = lane + DX_WAVE * h, rc = min(r, nefc - 1);
    const bool ok = r < nefc, fr = ok && r < c.nfric;
    ty[h] = ok ? (meta[rc] & 15) : DXR_CON;
    D[h] = ok ? Dp[rc] : 0.f;
    fl[h] = fr ? flp[rc] : 0.f;
    Rf[h] = fr ? Rfp[rc] : 0.f;
    ja[h] = ok ? jar[rc] : 0.f;
    jj[h] = 0.f;
#pragma unroll
    for (int d = 0; d < 30; d++) Jd[h][d] = 0.f;
    if (DX_WAVE * h < nefc)
      pgs_row_nz(c, ok ? r : -1, [&](int e, float v) {  // (v = 0 from lanes without a nonzero here)
#pragma unroll
        for (int d = 0; d < 30; d++) Jd[h][d] = d == e ? Jd[h][d] + v : Jd[h][d];
      });
  }
  auto rows_of = [&](const float (&mr)[30], float v) {  // (mr v) of this lane's row
    float y0 = 0.f, y1 = 0.f;
#pragma unroll
    for (int e = 0; e < 30; e += 2) {
      y0 = fmaf(mr[e], rl(v, e), y0);
      y1 = fmaf(mr[e + 1], rl(v, e + 1), y1);
    }
    return y0 + y1;
  };
  auto jt_force = [&]() {  // (J'f)_d of the rows' forces at the residuals ja
    float t[32];
#pragma unroll
    for (int d = 0; d < 32; d++) t[d] = 0.f;
#pragma unroll
    for (int h = 0; h < 2; h++) {
      if (DX_WAVE * h < nefc) {
        float f, hw;
        row_force(ty[h], D[h], fl[h], Rf[h], ja[h], f, hw);
#pragma unroll
        for (int d = 0; d < 30; d++) t[d] = fmaf(f, Jd[h][d], t[d]);
      }
    }
    const float w = wave_reduce_scatter32(t);  // component LANE >> 1
    const float wd = __int_as_float(__builtin_amdgcn_ds_bpermute(8 * (lane & 31), __float_as_int(w)));
    return dof ? wd : 0.f;
  };
  auto j_dir = [&](float v) {  // jj = J v, row by row in the row's lane
    float xs[30];
#pragma unroll
    for (int d = 0; d < 30; d++) xs[d] = rl(v, d);
#pragma unroll
    for (int h = 0; h < 2; h++) {
      float s0 = 0.f, s1 = 0.f;
      if (DX_WAVE * h < nefc) {
#pragma unroll
        for (int d = 0; d < 30; d += 2) {
          s0 = fmaf(Jd[h][d], xs[d], s0);
          s1 = fmaf(Jd[h][d + 1], xs[d + 1], s1);
        }
      }
      jj[h] = s0 + s1;
    }
  };
  float grad = ma - q0 - jt_force();
  float mg = rows_of(trow, grad);
  float dir = -mg, mdir = -grad;
  float gmg_old = wave_sum(grad * mg);
  int it = 0;
  for (; it < c.iterations; it++) {
    stage_count(c, CNT_NEWTON_IT);
    j_dir(dir);
    stage_mark(c, ST_JACVEC);
    // the exact line search (line_search<false, true>) on the row registers
    const float qa = wave_sum(dir * mdir), qb = wave_sum(dir * (ma - q0));
    float lo = 0.f, hi = -1.f, alpha = 0.f, g0 = 0.f;
    int ls = 0;
    for (; ls < 40; ls++) {
      float g = 0.f, hh = 0.f;
#pragma unroll
      for (int h = 0; h < 2; h++) {
        if (DX_WAVE * h < nefc) {
          float f, hw;
          row_force(ty[h], D[h], fl[h], Rf[h], ja[h] + alpha * jj[h], f, hw);
          g -= f * jj[h];
          hh += hw * jj[h] * jj[h];
        }
      }
      g = wave_sum(g) + qa * alpha + qb;
      hh = wave_sum(hh) + qa;
      if (ls == 0) g0 = g;
      if (fabsf(g) <= 1e-6f * fabsf(g0)) break;
      if (g < 0) lo = alpha; else hi = alpha;
      float next = hh > 0 ? alpha - g / hh : alpha + 1;
      if (hi >= 0 && (next <= lo || next >= hi)) next = 0.5f * (lo + hi);
      if (hi < 0 && next <= lo) next = lo + 1;
      if (fabsf(next - alpha) <= 1e-7f * fabsf(alpha)) break;
      alpha = next;
    }
    stage_count(c, CNT_LS_IT, min(ls + 1, 40));
    stage_mark(c, ST_NEWTON_LS);
    if (alpha == 0.f) break;
    x = fmaf(alpha, dir, x);
    ma = fmaf(alpha, mdir, ma);
    const float mg_old = mg;
#pragma unroll
    for (int h = 0; h < 2; h++) ja[h] = fmaf(alpha, jj[h], ja[h]);
    // the decrease along the line, -alpha g0 / 2 (solve_cg)
    const float impr = -0.5f * scale * alpha * g0;
    grad = ma - q0 - jt_force();
    const float gn = sqrtf(wave_sum(grad * grad)) * scale;
    mg = rows_of(trow, grad);
    stage_mark(c, ST_NEWTON_GRAD);
    if (impr < tol || gn < tol) {
      it++;
      break;
    }
    const float num = wave_sum(grad * (mg - mg_old)), gmg = wave_sum(grad * mg);
    const float beta = fmaxf(0.f, num / fmaxf(1e-15f, gmg_old));
    gmg_old = gmg;
    const float di = -mg + beta * dir;
    const bool restart = !(wave_sum(grad * di) < 0.f);  // not a descent direction
    dir = restart ? -mg : di;
    mdir = restart ? -grad : fmaf(beta, mdir, -grad);
    // (the recurrences hold only as far as M M^-1 = I: M qacc and M dir exactly on a
    // restart and every 8 iterations, as solve_cg)
    if (restart || (it & 7) == 7) {
      ma = rows_of(mrow, x);
      mdir = rows_of(mrow, dir);
    }
  }
  if (dof) { qacc[lane] = x; Ma[lane] = ma; }
#pragma unroll
  for (int h = 0; h < 2; h++) {
    const int r = lane + DX_WAVE * h;
    if (r < nefc) jar[r] = ja[h];
  }
  if (lane == 0) c.I[I_NITER] = it;
  SYNC();
}
// [3P] MuJoCo's primal CG (mj_solCG), <option solver="CG">: the Newton solver's cost,
// warm start and exact line search with Polak-Ribiere directions preconditioned by M
// (Mgrad = M^-1 grad through the matrix-core Cholesky of M), and the same convergence
// tests -- with the improvement taken from the line search (-alpha g0 / 2) rather than
// as a difference of fp32 costs.  A non-descent direction restarts along -Mgrad.  Not
// the default (the reference's scenes run Newton); oracle: dx_oracle.c solve_cg.
template <class Ctx>
__device__ __forceinline__ void solve_cg(const Ctx& c, float scale, float tol) {
  const int nv = c.nv;
  float* qacc = c.f(c.L.qacc);
  float* Ma = c.f(c.L.v1);
  float* grad = c.f(c.L.v2);
  float* dir = c.f(c.L.v3);
  float* Mg_old = c.f(c.L.v5);  // the warm start copy is dead now
  float* Mg = c.f(c.L.cgv);
  float* jar = c.f(c.L.efc_jar);
  const float* M = c.f(c.L.M);
  const float* qs = c.f(c.L.qfrc_smooth);
  float* T = c.f(c.L.H);
  // M^-1 once per solve (nv <= 30: the sweep's inverse, packed in the Newton Hessian's
  // region, which CG does not use), then one product per iteration; larger nv solve each
  // time (the LDS Cholesky)
  const bool inv = DX_SWEEP && nv <= 30;
  float trow[30];  // lane i: row i of M^-1 in registers (mrow_load), one product per iteration
  if (inv) {
    mfma_sweep_inverse30(M, nv, T);
    mrow_load(T, nv, trow);
  }
  auto minv = [&]() {
    if (inv) {
      mat_vec_rows(trow, grad, Mg, nv);
      SYNC();
    } else {
      for (int i = LANE; i < nv; i += DX_WAVE) Mg[i] = grad[i];
      SYNC();
      chol_solve(M, nv, Mg, T);
    }
  };
  // J's rows dense in registers (lane r: rows r and 64 + r, up to 128 rows, nv <= 30):
  // J dir is then one FMA per dof with dir broadcast from LDS, and J'f a reduce-scatter of
  // every lane's f_r J_r over the wave (wave_reduce_scatter32) -- no contact-frame passes,
  // no LDS atomics.  (Other sizes keep jac_vec / jac_t_force.)
  const int nefc = c.I[I_NEFC];
  const bool jreg = DX_SWEEP && nv <= 30 && nefc <= 2 * DX_WAVE;
  const int lane = LANE;
  float Jd[2][30];
#pragma unroll
  for (int d = 0; d < 30; d++) Jd[0][d] = Jd[1][d] = 0.f;
  if (jreg) {
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const int r = lane + DX_WAVE * h;
      if (DX_WAVE * h < nefc)
        pgs_row_nz(c, r < nefc ? r : -1, [&](int e, float v) {  // (v = 0 from lanes without a nonzero here)
#pragma unroll
          for (int d = 0; d < 30; d++) Jd[h][d] = d == e ? Jd[h][d] + v : Jd[h][d];
        });
    }
  }
  auto jdir = [&](const float* x, float* out) {  // out[r] = J_r x
    float xs[30];
#pragma unroll
    for (int d = 0; d < 30; d++) xs[d] = x[min(d, nv - 1)];  // (uniform addresses: broadcast reads)
#pragma unroll
    for (int h = 0; h < 2; h++) {
      if (DX_WAVE * h < nefc) {
        float s0 = 0.f, s1 = 0.f;
#pragma unroll
        for (int d = 0; d < 30; d += 2) {
          s0 = fmaf(Jd[h][d], d < nv ? xs[d] : 0.f, s0);
          s1 = fmaf(Jd[h][d + 1], d + 1 < nv ? xs[d + 1] : 0.f, s1);
        }
        const int r = lane + DX_WAVE * h;
        if (r < nefc) out[r] = s0 + s1;
      }
    }
    SYNC();
  };
  const int* meta = (const int*)c.f(c.L.efc_meta);
  const float* Dp = c.f(c.L.efc_D);
  const float* flp = c.f(c.L.efc_fl);
  const float* Rfp = c.f(c.L.efc_Rf);
  auto jtf = [&](float* out) {  // out = J'f, f the rows' forces at jar
    float t[32];
#pragma unroll
    for (int d = 0; d < 32; d++) t[d] = 0.f;
#pragma unroll
    for (int h = 0; h < 2; h++) {
      if (DX_WAVE * h < nefc) {
        const int r = lane + DX_WAVE * h, rc = min(r, nefc - 1);
        const bool fr = r < c.nfric;
        float f, hw;
        row_force(meta[rc] & 15, Dp[rc], fr ? flp[rc] : 0.f, fr ? Rfp[rc] : 0.f, jar[rc], f, hw);
        f = r < nefc ? f : 0.f;
#pragma unroll
        for (int d = 0; d < 30; d++) t[d] = fmaf(f, Jd[h][d], t[d]);
      }
    }
    const float w = wave_reduce_scatter32(t);  // component LANE >> 1
    const float wd = __int_as_float(__builtin_amdgcn_ds_bpermute(8 * (lane & 31), __float_as_int(w)));
    if (lane < nv) out[lane] = wd;
    SYNC();
  };
  int it = 0;
  if (jreg) jtf(grad);
  else jac_t_force(c, grad);  // grad <- J^T f
  for (int i = LANE; i < nv; i += DX_WAVE) grad[i] = Ma[i] - qs[i] - grad[i];
  SYNC();
  minv();
  float gmg = 0;
  for (int i = LANE; i < nv; i += DX_WAVE) {
    dir[i] = -Mg[i];
    gmg += grad[i] * Mg[i];
  }
  float gmg_old = wave_sum(gmg);
  // M dir by recurrence instead of a product per iteration: dir = -M^-1 grad + beta dir_old
  // gives M dir = -grad + beta M dir_old (-grad on a restart)
  float* Mdir = c.f(c.L.v4);
  for (int i = LANE; i < nv; i += DX_WAVE) Mdir[i] = -grad[i];
  SYNC();
  for (; it < c.iterations; it++) {
    stage_count(c, CNT_NEWTON_IT);
    int changed = 0;
    float g0 = 0.f;
    float alpha;
    if (jreg) {
      jdir(dir, c.f(c.L.efc_jv));
      stage_mark(c, ST_JACVEC);
      alpha = line_search<false, true, false, true>(c, qacc, Ma, dir, &changed, &g0);
    } else {
      alpha = line_search<false, true>(c, qacc, Ma, dir, &changed, &g0);
    }
    stage_mark(c, ST_NEWTON_LS);
    if (alpha == 0.f) break;
    const float* jvd = c.f(c.L.efc_jv);
    for (int i = LANE; i < nv; i += DX_WAVE) {
      qacc[i] += alpha * dir[i];
      Ma[i] += alpha * Mdir[i];
      Mg_old[i] = Mg[i];
    }
    for (int r = LANE; r < c.I[I_NEFC]; r += DX_WAVE) jar[r] += alpha * jvd[r];
    SYNC();
    // the decrease along the line, -alpha g0 / 2 (exact for a quadratic segment): the
    // difference of two fp32 costs drowns in rounding long before CG's slow tail ends
    const float impr = -0.5f * scale * alpha * g0;
    if (jreg) jtf(grad);
    else jac_t_force(c, grad);
    float gn = 0;
    for (int i = LANE; i < nv; i += DX_WAVE) {
      grad[i] = Ma[i] - qs[i] - grad[i];
      gn += grad[i] * grad[i];
    }
    gn = sqrtf(wave_sum(gn)) * scale;
    SYNC();
    minv();
    stage_mark(c, ST_NEWTON_GRAD);
    if (impr < tol || gn < tol) {
      it++;
      break;
    }
    float num = 0;
    gmg = 0;
    for (int i = LANE; i < nv; i += DX_WAVE) {
      num += grad[i] * (Mg[i] - Mg_old[i]);
      gmg += grad[i] * Mg[i];
    }
    num = wave_sum(num);
    gmg = wave_sum(gmg);
    const float beta = fmaxf(0.f, num / fmaxf(1e-15f, gmg_old));
    gmg_old = gmg;
    float slope = 0;
    for (int i = LANE; i < nv; i += DX_WAVE) {
      const float di = -Mg[i] + beta * dir[i];
      slope += grad[i] * di;
      dir[i] = di;
    }
    // not a descent direction (fp32 line searches are exact to 1e-6): restart along -Mgrad
    const bool restart = !(wave_sum(slope) < 0.f);
    for (int i = LANE; i < nv; i += DX_WAVE) {
      if (restart) dir[i] = -Mg[i];
      Mdir[i] = restart ? -grad[i] : fmaf(beta, Mdir[i], -grad[i]);
    }
    SYNC();
    // The recurrences hold only as far as M Mg = grad does, i.e. to the rounding of the
    // fp32 M^-1: M qacc and M dir exactly on a restart and every 8 iterations, so the
    // gradient (and CG's stopping point) does not drift from the cost's
    if (restart || (it & 7) == 7) {
      mat_vec(M, qacc, Ma, nv);
      mat_vec(M, dir, Mdir, nv);
      SYNC();
    }
  }
  if (LANE == 0) c.I[I_NITER] = it;
  SYNC();
}

// Entry (r, LANE) of J (lane d: dof d, 0 past nv), from the rows' compact forms (jac_rows).
template <class Ctx>
__device__ __forceinline__ float pgs_jrow(const Ctx& c, int r) {
  const DevModel& m = c.mdl();
  const int nv = c.nv;
  const int mt = ((const int*)c.f(c.L.efc_meta))[r], type = mt & 15, aux = (mt >> 4) & 15, id = mt >> 8;
  float v = 0.f;
  if (LANE < nv) {
    const int d = LANE;
    if (type == DXR_FRIC) {
      v = d == id ? 1.f : 0.f;
    } else if (type == DXR_LIMJ) {
      v = d == id ? (aux ? -1.f : 1.f) : 0.f;
    } else if (type == DXR_LIMT) {
      const float tj = m.tendon_J[id * nv + d];
      v = aux ? -tj : tj;
    } else {
      const float* rc = c.f(c.L.con) + DX_CON_STRIDE * id;
      const uint64_t sup = (uint64_t)(uint32_t)__float_as_int(rc[18]) | ((uint64_t)(uint32_t)__float_as_int(rc[19]) << 32);
      const uint64_t bit = 1ull << d;
      const int q = __popcll(sup & (bit - 1));
      if ((sup & bit) && q < DX_DOFMAX) {
        const float* cv = c.f(c.L.cj_val) + id * 3 * DX_DOFMAX + q;
        v = cv[0];
        if (type == DXR_CON) {
          const int k = 1 + (aux >> 1);
          v += rc[15 + k] * ((aux & 1) ? -1.f : 1.f) * cv[k * DX_DOFMAX];
        }
      }
    }
  }
  return v;
}
// Dense row r of J into Jd (LDS)
template <class Ctx>
__device__ __forceinline__ void pgs_row(const Ctx& c, int r, float* Jd) {
  const float v = pgs_jrow(c, r);
  if (LANE < c.nv) Jd[LANE] = v;
  SYNC();
}

#ifndef DX_PGS_NB
#define DX_PGS_NB 3  // PGS register blocks of 64 rows (AR's diagonal blocks, one column per lane)
#endif
#define DX_PGS_AR 64
#ifndef DX_PGS_NB_TIER
#if defined(DX_TIER_HI)
#define DX_PGS_NB_TIER 3
#else
#define DX_PGS_NB_TIER 2
#endif
#endif
// Visit the nonzeros (e, v) of constraint row k (k < 0: none) from the row's compact form
// (jac_rows / pgs_jrow): one dof (friction loss, joint limit), a tendon's dofs, or a
// contact row's support dofs.  k may differ by lane (then e and v do too) or be uniform.
template <class Ctx, class F>
__device__ __forceinline__ void pgs_row_nz(const Ctx& c, int k, F&& add) {
  const DevModel& m = c.mdl();
  const int nv = c.nv;
  const int mt = k >= 0 ? ((const int*)c.f(c.L.efc_meta))[k] : 0;
  const int type = mt & 15, aux = (mt >> 4) & 15, id = mt >> 8;
  const bool on = k >= 0;
  const bool con = on && (type == DXR_CON || type == DXR_CONFL);
  const float* rc = c.f(c.L.con) + DX_CON_STRIDE * (con ? id : 0);
  uint64_t sup = con ? ((uint64_t)(uint32_t)__float_as_int(rc[18]) | ((uint64_t)(uint32_t)__float_as_int(rc[19]) << 32)) : 0ull;
  const int kk = 1 + (aux >> 1);
  const float mu = type == DXR_CON ? rc[15 + kk] * ((aux & 1) ? -1.f : 1.f) : 0.f;
  const float* cv = c.f(c.L.cj_val) + (con ? id : 0) * 3 * DX_DOFMAX;
  const bool one = on && (type == DXR_FRIC || type == DXR_LIMJ);
  if (__any(one)) add(one ? id : 0, one ? (type == DXR_LIMJ && aux ? -1.f : 1.f) : 0.f);
  if (c.nlimt > 0 && __any(on && type == DXR_LIMT))
    for (int e = 0; e < nv; e++) {
      const float tj = m.tendon_J[(on && type == DXR_LIMT ? id : 0) * nv + e];
      add(e, on && type == DXR_LIMT ? (aux ? -tj : tj) : 0.f);
    }
#pragma unroll 1
  for (int q = 0; q < DX_DOFMAX; q++) {  // (not unrolled: the caller's accumulators stay live)
    if (!__any(sup != 0ull)) break;
    const int e = sup ? (int)__builtin_ctzll(sup) : 0;
    const float v = sup ? cv[q] + mu * cv[kk * DX_DOFMAX + q] : 0.f;
    sup &= sup - 1;
    if (__any(v != 0.f)) add(e, v);
  }
}
// P_k = G' J_k' for constraint row k of this lane (k < 0: zero), nv <= 30, where G (a
// packed lower triangle with its diagonal in LDS, mfma_chol_factor30) is the Cholesky
// factor of M^-1: y[d] = sum over the row's nonzeros (e, v) of G[e][d] v (d <= e), so
// that P_k . P_r = J_k M^-1 J_r' = A[k][r].
template <class Ctx>
__device__ __forceinline__ void pgs_p_row(const Ctx& c, int k, const float* G, float (&y)[30]) {
  const int nv = c.nv;
#pragma unroll
  for (int d = 0; d < 30; d++) y[d] = 0.f;
  pgs_row_nz(c, k, [&](int e, float v) {
#pragma unroll
    for (int d = 0; d < 30; d++) y[d] = fmaf(G[ti(e) + min(d, e)], d <= e && d < nv ? v : 0.f, y[d]);
  });
}
// Lane d: (G' J_r')[d] for a uniform row r (the tail rows past the register blocks)
template <class Ctx>
__device__ __forceinline__ float pgs_p_lane(const Ctx& c, int r, const float* G) {
  const int d = LANE, nv = c.nv;
  float p = 0.f;
  pgs_row_nz(c, r, [&](int e, float v) { p = fmaf(G[ti(e) + min(d, e)], d <= e && d < nv ? v : 0.f, p); });
  return p;
}
// f(std::integral_constant<int, I>) for I in the sequence, unrolled: a register array
// indexed by I stays in registers
template <class F, int... I>
__device__ __forceinline__ void static_for(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
// PGS on MuJoCo's own form (mj_solPGS on efc_AR) for nv <= 30, solve_pgs's path up to
// DX_PGS_NB x 64 rows (+ a tail of 64).  AR = J M^-1 J' + R is held in registers in
// diagonal blocks of 64 rows, lane k holding column k of its block (A[B][r] = AR[64B +
// r][64B + k], AR is symmetric); the coupling between blocks is carried in "whitened"
// force space.  With G the Cholesky factor of M^-1 (mfma_chol_factor30 over the sweep's
// inverse) and P_k = G' J_k' (lane k of block B holds its row's P, 30 registers), AR =
// P P' + R, and the residual of row k is res_k = (AR f)_k + b_k = P_k . w + R_k f_k + b_k
// with w = sum over all rows of f_r P_r and b = J qacc_smooth - aref.
//  * Forming: P by the rows' compact forms (pgs_p_row), each diagonal block P_B P_B' on
//    the matrix cores (pgs_gram64: 15-60 v_mfma_f32_32x32x2_f32) -- the batched J M^-1 J'
//    contraction;
//  * a block's sweep starts from its residuals recomputed from w (w reduce-scattered
//    over the lanes from every lane's f P, wave_reduce_scatter32, then 30 readlanes and
//    FMAs) -- the Gauss-Seidel sweep in row order, with no matrix-free pass through J,
//    M^-1 and J';
//  * a row update runs in the row's own lane: every lane projects its own candidate
//    (fmed3 of f - res / AR_kk onto the row's box [-floss, floss] or [0, inf); padding rows
//    past nefc have the box [0, 0]), the row's change is one readlane, and every lane's
//    residual takes one FMA with its AR entry: 7 instructions, no reduction and no
//    per-row broadcast of the row's constants on the chain from one row to the next;
//  * the sweep's dual-cost decrease sum_r -(AR_rr df_r^2 / 2 + df_r res_r) from each lane's
//    force change and its residual at its own update (snapshot), one wave sum per sweep;
//  * rows past the blocks (the tail) run one at a time in w space: lane d holds w[d] and
//    (G' J_r')[d] (pgs_p_lane), res_r = wave sum + R_r f_r + b_r, w += df P_r;
//  * at the end qacc = qacc_smooth + M^-1 J'f = qacc_smooth + G w.
// Rows visited, projections and stopping test are the oracle's (dx_oracle.c solve_pgs).
template <int NB, class Ctx>
__device__ __forceinline__ void solve_pgs_ar(const Ctx& c, float scale, float tol, float* T) {
  const int nv = c.nv, nefc = c.I[I_NEFC];
  float* qacc = c.f(c.L.qacc);
  const float* a0 = c.f(c.L.qacc_smooth);
  float* f = c.f(c.L.efc_jv);
  float* jar = c.f(c.L.efc_jar);
  const int* meta = (const int*)c.f(c.L.efc_meta);
  const float* D = c.f(c.L.efc_D);
  const float* fl = c.f(c.L.efc_fl);
  const float* aref = c.f(c.L.efc_aref);
  const int nb = min(NB, (nefc + DX_PGS_AR - 1) / DX_PGS_AR);  // blocks in use
  const int ntail = max(0, nefc - NB * DX_PGS_AR);
  jac_vec(c, a0, jar);       // J qacc_smooth (the warm start's residuals were consumed): b = jar - aref
  mfma_chol_factor30(T, nv);  // G over M^-1
  const float* G = T;
  auto box = [&](int k, float& lo, float& hi) {
    const int kc = min(k, nefc - 1);
    const bool fr = (meta[kc] & 15) == DXR_FRIC;
    hi = k >= nefc ? 0.f : fr ? fl[kc] : __builtin_inff();
    lo = fr && k < nefc ? -hi : 0.f;
  };
  constexpr auto blocks = std::make_integer_sequence<int, NB>{};
  constexpr auto rows = std::make_integer_sequence<int, DX_PGS_AR>{};
  // Per lane and block: its row's P, its column of AR scaled by 1 / AR_kk (A'), and the
  // row's state in the scaled form the row update's chain needs: res' = res / AR_kk, and
  // the box relative to the force, lof = lo - f, hif = hi - f, so that the force change of
  // a row is dl = med3(-res', lof, hif) (f - res / AR_kk projected on [lo, hi], minus f).
  const int lane = LANE;
  float P[NB][30], A[NB][DX_PGS_AR];
  float lof[NB], hif[NB], lob[NB], res[NB], rs[NB], bb[NB], rk[NB], dgv[NB], idg[NB];
  static_for([&](auto Bc) {
    constexpr int B = Bc.value;
    const int k = DX_PGS_AR * B + lane;
    const bool in = k < nefc;
    const int kc = min(k, nefc - 1);
    rk[B] = in ? 1.0f / D[kc] : 0.f;
    const float f0 = in ? f[kc] : 0.f;
    bb[B] = in ? jar[kc] - aref[kc] : 0.f;
    float l, h;
    box(k, l, h);
    lob[B] = l;
    lof[B] = l - f0;
    hif[B] = h - f0;
    res[B] = 0.f;
    rs[B] = 0.f;
    if (B < nb) {
      pgs_p_row(c, in ? k : -1, G, P[B]);
      pgs_gram64(P[B], rk[B], nefc > DX_PGS_AR * B + 32, A[B]);
    } else {
#pragma unroll
      for (int d = 0; d < 30; d++) P[B][d] = 0.f;
      static_for([&](auto K) { A[B][K.value] = 0.f; }, rows);
    }
    float dg = 1.f;  // AR_kk, this lane's diagonal entry (1 on a padding row)
    static_for([&](auto K) { dg = lane == K.value ? A[B][K.value] : dg; }, rows);
    dg = in ? dg : 1.f;
    dgv[B] = dg;
    idg[B] = 1.0f / dg;
    static_for([&](auto K) { A[B][K.value] *= idg[B]; }, rows);
  }, blocks);
  float ardt = 1.f;  // lane t: AR of tail row NB x 64 + t on the diagonal
  for (int t = 0; t < ntail; t++) {
    const int r = NB * DX_PGS_AR + t;
    const float p = pgs_p_lane(c, r, G);
    const float s = wave_sum(p * p) + 1.0f / D[r];
    ardt = LANE == t ? s : ardt;
  }
  stage_mark(c, ST_NEWTON_HESS);
  // w (lane d: w[d]) from every row's current force; wt, the tail rows' part, is kept
  // current by their updates
  float wt = 0.f, wl = 0.f;
  auto wsum = [&]() {
    float t[32];
#pragma unroll
    for (int d = 0; d < 32; d++) t[d] = 0.f;
    static_for([&](auto Bc) {
      if (Bc.value < nb) {
        const float fk = lob[Bc.value] - lof[Bc.value];  // this lane's row's force
#pragma unroll
        for (int d = 0; d < 30; d++) t[d] = fmaf(fk, P[Bc.value][d], t[d]);
      }
    }, blocks);
    const float r = wave_reduce_scatter32(t);  // component LANE >> 1
    const float wd = __int_as_float(__builtin_amdgcn_ds_bpermute(8 * (LANE & 31), __float_as_int(r)));
    wl = (LANE < nv ? wd : 0.f) + wt;
  };
  auto dotw = [&](const float (&p)[30]) {
    float s0 = 0.f, s1 = 0.f;
#pragma unroll
    for (int d = 0; d < 30; d += 2) {
      s0 = fmaf(p[d], rl(wl, d), s0);
      s1 = fmaf(p[d + 1], rl(wl, d + 1), s1);
    }
    return s0 + s1;
  };
  // one row update, in the row's lane q (q static: a register name of A[B]).  The chain
  // from one row to the next is med3 -> readlane -> fma.  A lane's box (lof, hif) changes
  // only at its own row, which a sweep visits once, so the row's change is kept (dsv) and
  // the box moves after the block's sweep; its residual at the update is kept too (snap).
#define DX_PGS_ROWL(q, Acol, rsv, lofv, hifv, dsv, snap)                \
  {                                                                     \
    const float dla = __builtin_amdgcn_fmed3f(-rsv, lofv, hifv);        \
    const float dl = rl(dla, q);                                        \
    const bool me = lg == (q);                                          \
    dsv = me ? dla : dsv;                                               \
    snap = me ? rsv : snap;                                             \
    rsv = fmaf(dl, Acol[q], rsv);                                       \
  }
  constexpr auto groups = std::make_integer_sequence<int, DX_PGS_AR / 8>{};
  constexpr auto eight = std::make_integer_sequence<int, 8>{};
  int it = 0;
  for (; it < c.iterations;) {
    stage_count(c, CNT_NEWTON_IT);
    float il = 0.f;  // this lane's rows' dual-cost decrease
    float impr = 0.f;
    static_for([&](auto Bc) {
      constexpr int B = Bc.value;
      if (B < nb) {
        // (profiling: the residuals count as newton_grad, the row updates as
        // newton_linesearch, the formation above as newton_hessian)
        if (nb > 1 || ntail > 0 || it == 0) {  // (one block alone keeps its residuals current)
          wsum();
          res[B] = (dotw(P[B]) + bb[B] + rk[B] * (lob[B] - lof[B])) * idg[B];
          stage_mark(c, ST_NEWTON_GRAD);
        }
        float df = 0.f;  // this lane's row's force change in the sweep
        static_for([&](auto Gc) {
          if (DX_PGS_AR * B + 8 * Gc.value < nefc) {
            // (the lane id laundered per group: the compiler would otherwise hoist all 64
            // lane == q masks out of the sweep loop and spill them)
            int lg = lane;
            asm volatile("" : "+v"(lg));
            static_for([&](auto Q) { DX_PGS_ROWL(8 * Gc.value + Q.value, A[B], res[B], lof[B], hif[B], df, rs[B]) },
                       eight);
          }
        }, groups);
        lof[B] -= df;
        hif[B] -= df;
        // -(AR_kk df^2 / 2 + df res) with res = AR_kk res' at the row's update
        il -= df * dgv[B] * fmaf(0.5f, df, rs[B]);
        stage_mark(c, ST_NEWTON_LS);
      }
    }, blocks);
    if (ntail) {
      wsum();
      stage_mark(c, ST_NEWTON_GRAD);
      for (int t = 0; t < ntail; t++) {
        const int r = NB * DX_PGS_AR + t;
        const float p = pgs_p_lane(c, r, G);
        const float fo = f[r];
        const float rr = wave_sum(p * wl) + (jar[r] - aref[r]) + fo / D[r];
        const float ar = rl(ardt, t);
        float l, h;
        box(r, l, h);
        const float fn = __builtin_amdgcn_fmed3f(fo - rr / ar, l, h);
        const float dl = fn - fo;
        if (dl != 0.f) {
          wl = fmaf(dl, p, wl);
          wt = fmaf(dl, p, wt);
          if (LANE == 0) f[r] = fn;
          impr -= 0.5f * ar * dl * dl + dl * rr;
        }
        SYNC();
      }
      stage_mark(c, ST_NEWTON_LS);
    }
    impr += wave_sum(il);
    it++;
    if (scale * impr < tol) break;
  }
#undef DX_PGS_ROWL
  // qacc = qacc_smooth + G w (lane d: sum over e <= d of G[d][e] w[e])
  wsum();
  {
    const int d = min(LANE, nv - 1);
    float s0 = 0.f, s1 = 0.f;
#pragma unroll
    for (int e = 0; e < 30; e += 2) {
      s0 = fmaf(e <= d ? G[ti(d) + min(e, d)] : 0.f, rl(wl, min(e, 29)), s0);
      s1 = fmaf(e + 1 <= d ? G[ti(d) + min(e + 1, d)] : 0.f, rl(wl, min(e + 1, 29)), s1);
    }
    SYNC();
    if (LANE < nv) qacc[LANE] = a0[LANE] + (s0 + s1);
  }
  // the forces, as residuals whose primal force is f_r
  static_for([&](auto Bc) {
    const int k = DX_PGS_AR * Bc.value + lane;
    const float fk = lob[Bc.value] - lof[Bc.value];
    if (k < nefc) {
      f[k] = fk;
      jar[k] = -fk / D[k];
    }
  }, blocks);
  for (int r = NB * DX_PGS_AR + LANE; r < nefc; r += DX_WAVE) jar[r] = -f[r] / D[r];
  if (LANE == 0) c.I[I_NITER] = it;
  SYNC();
}
// [3P] MuJoCo's PGS (mj_solPGS), <option solver="PGS">: projected Gauss-Seidel on the
// dual, min_f 0.5 f'(A + R) f + f'b with A = J M^-1 J' and b = J qacc_smooth - aref;
// friction-loss rows boxed to +-floss, limit and pyramidal contact rows f >= 0, rows in
// order, each f_r -= res_r / AR_rr and projected.  Matrix-free: qacc = qacc_smooth +
// M^-1 J'f is kept current, so res_r = J_r qacc - aref_r + R_r f_r and no nefc x nefc
// matrix is held in LDS; M^-1 J_r' is one product with M^-1 (the sweep's inverse, nv <=
// 30, as CG) or one Cholesky solve, only for a row whose force changed.  Warm start: the
// primal forces at qacc_warmstart, kept when their dual cost is below zero's.  Stops
// after `iterations` sweeps or when a sweep's scaled dual-cost decrease is below the
// tolerance.  The forces go back as residuals jar_r = -R_r f_r, whose primal force
// (row_cost) is f_r, so qfrc_constraint and the sensors read them unchanged.  Oracle:
// dx_oracle.c solve_pgs.  Serial over rows: a scene option, not the reference's path.
template <class Ctx>
__device__ __forceinline__ void solve_pgs(const Ctx& c, float scale, float tol) {
  const int nv = c.nv, nefc = c.I[I_NEFC];
  float* qacc = c.f(c.L.qacc);
  const float* a0 = c.f(c.L.qacc_smooth);
  float* g = c.f(c.L.v2);
  float* Jd = c.f(c.L.v3);
  float* u = c.f(c.L.cgv);
  float* f = c.f(c.L.efc_jv);
  float* jar = c.f(c.L.efc_jar);  // the warm start's residuals, then AR's diagonal
  float* ard = jar;
  const int* meta = (const int*)c.f(c.L.efc_meta);
  const float* D = c.f(c.L.efc_D);
  const float* fl = c.f(c.L.efc_fl);
  const float* Rf = c.f(c.L.efc_Rf);
  const float* aref = c.f(c.L.efc_aref);
  const float* M = c.f(c.L.M);
  float* T = c.f(c.L.H);
  const bool inv = DX_SWEEP && nv <= 30;
  if (inv) mfma_sweep_inverse30(M, nv, T);
  auto minv = [&](const float* x, float* y) {
    if (inv) {
      mat_vec(T, x, y, nv);
      SYNC();
    } else {
      for (int i = LANE; i < nv; i += DX_WAVE) y[i] = x[i];
      SYNC();
      chol_solve(M, nv, y, T);
    }
  };
  // warm start: jar holds J qacc_warmstart - aref (solve); g = J'f, u = M^-1 g
  float dc = 0.f;
  for (int r = LANE; r < nefc; r += DX_WAVE) {
    const bool fr = r < c.nfric;
    float fo, hw;
    row_force(meta[r] & 15, D[r], fr ? fl[r] : 0.f, fr ? Rf[r] : 0.f, jar[r], fo, hw);
    f[r] = fo;
    dc += 0.5f * fo * fo / D[r] - fo * aref[r];
  }
  jac_t_force(c, g);
  minv(g, u);
  for (int i = LANE; i < nv; i += DX_WAVE) dc += 0.5f * g[i] * u[i] + g[i] * a0[i];
  const bool keep = wave_sum(dc) < 0.f;
  for (int i = LANE; i < nv; i += DX_WAVE) qacc[i] = keep ? a0[i] + u[i] : a0[i];
  if (!keep)
    for (int r = LANE; r < nefc; r += DX_WAVE) f[r] = 0.f;
  SYNC();
  if (inv) {
    // (the generic kernel and the mid tier, within two waves' VGPRs, hold two blocks; the
    // overflow tier runs one wave per SIMD)
    constexpr int NB = Ctx::is_spec ? DX_PGS_NB : DX_PGS_NB_TIER;
    if (nefc <= NB * DX_PGS_AR + DX_WAVE) {
      solve_pgs_ar<NB>(c, scale, tol, T);
      return;
    }
    // nv <= 30: the sweep's M^-1 row of dof d in lane d's registers, qacc[d] in lane d,
    // J_r built in registers (lane d: entry d), so a row update is a DPP dot product, a
    // few scalars and, for a changed force, M^-1 J_r' from 30 readlanes -- no LDS round
    // trip on the chain from one row to the next
    float mi[30];
    const int d = min(LANE, nv - 1);
#pragma unroll
    for (int k = 0; k < 30; k++) {
      const int kc = min(k, nv - 1);
      const float t = T[ti(max(d, kc)) + min(d, kc)];
      mi[k] = LANE < nv && k < nv ? t : 0.f;
    }
    float qa = LANE < nv ? qacc[LANE] : 0.f;
    auto minv_row = [&](float jr) {
      float u0 = 0.f, u1 = 0.f;
#pragma unroll
      for (int k = 0; k < 30; k += 2) {
        u0 = fmaf(mi[k], rl(jr, k), u0);
        u1 = fmaf(mi[k + 1], rl(jr, k + 1), u1);
      }
      return u0 + u1;
    };
    for (int r = 0; r < nefc; r++) {
      const float jr = pgs_jrow(c, r);
      const float sr = wave_sum(jr * minv_row(jr));
      if (LANE == 0) ard[r] = sr + 1.0f / D[r];
    }
    SYNC();
    int it = 0;
    for (; it < c.iterations;) {
      stage_count(c, CNT_NEWTON_IT);
      float impr = 0.f;
      for (int r = 0; r < nefc; r++) {
        const float jr = pgs_jrow(c, r);
        const int ty = meta[r] & 15;
        const float fo = f[r], ar = ard[r], ra = aref[r], dr = D[r], fr = ty == DXR_FRIC ? fl[r] : 0.f;
        const float res = wave_sum(jr * qa) - ra + fo / dr;
        float fn = fo - res / ar;
        fn = ty == DXR_FRIC ? fminf(fr, fmaxf(-fr, fn)) : fmaxf(fn, 0.f);
        const float dl = fn - fo;
        if (dl != 0.f) {
          qa = fmaf(dl, minv_row(jr), qa);
          if (LANE == 0) f[r] = fn;
          impr -= 0.5f * ar * dl * dl + dl * res;
        }
      }
      it++;
      if (scale * impr < tol) break;
    }
    if (LANE < nv) qacc[LANE] = qa;
    for (int r = LANE; r < nefc; r += DX_WAVE) jar[r] = -f[r] / D[r];
    if (LANE == 0) c.I[I_NITER] = it;
    SYNC();
    return;
  }
  // AR's diagonal: J_r M^-1 J_r' + R_r
  for (int r = 0; r < nefc; r++) {
    pgs_row(c, r, Jd);
    minv(Jd, u);
    const float s = wave_sum(LANE < nv ? Jd[LANE] * u[LANE] : 0.f);
    if (LANE == 0) ard[r] = s + 1.0f / D[r];
  }
  SYNC();
  int it = 0;
  for (; it < c.iterations;) {
    stage_count(c, CNT_NEWTON_IT);
    float impr = 0.f;
    for (int r = 0; r < nefc; r++) {
      pgs_row(c, r, Jd);
      const float jq = wave_sum(LANE < nv ? Jd[LANE] * qacc[LANE] : 0.f);
      const float fo = f[r], ar = ard[r];
      const float res = jq - aref[r] + fo / D[r];
      float fn = fo - res / ar;
      if ((meta[r] & 15) == DXR_FRIC) fn = fminf(fl[r], fmaxf(-fl[r], fn));
      else fn = fmaxf(fn, 0.f);
      const float dl = fn - fo;
      if (dl != 0.f) {
        minv(Jd, u);
        if (LANE < nv) qacc[LANE] += dl * u[LANE];
        if (LANE == 0) f[r] = fn;
        impr -= 0.5f * ar * dl * dl + dl * res;
        SYNC();
      }
    }
    it++;
    if (scale * impr < tol) break;
  }
  // the forces as residuals whose primal force is f_r
  for (int r = LANE; r < nefc; r += DX_WAVE) jar[r] = -f[r] / D[r];
  if (LANE == 0) c.I[I_NITER] = it;
  SYNC();
}

template <class Ctx>
__device__ __forceinline__ void solve(const Ctx& c) {
  const DevModel& m = c.mdl();
  int nv = c.nv;
  float* qacc = c.f(c.L.qacc);
  float* a0 = c.f(c.L.qacc_smooth);
  float* ws = c.f(c.L.v5);  // warmstart copy held in v5 by the caller
  float* Ma = c.f(c.L.v1);
  float* grad = c.f(c.L.v2);
  float* dir = c.f(c.L.v3);
  const float* qs = c.f(c.L.qfrc_smooth);
  int nefc = c.I[I_NEFC];
  if (nefc == 0) {
    for (int i = LANE; i < nv; i += DX_WAVE) qacc[i] = a0[i];
    if (LANE == 0) c.I[I_NITER] = 0;
    SYNC();
    return;
  }
  float scale = 1.0f / (m.meaninertia * (float)max(1, nv));
  float tol = fmaxf(m.tolerance, 1e-9f);
  // warm start vs smooth.  M qacc_smooth = qfrc_smooth, so the smooth candidate needs
  // no M product and has a zero Gauss term: only J qacc_smooth (into efc_jv).
  float* jar = c.f(c.L.efc_jar);
  float* jvs = c.f(c.L.efc_jv);
  const float* aref = c.f(c.L.efc_aref);
  for (int i = LANE; i < nv; i += DX_WAVE) qacc[i] = ws[i];
  SYNC();
  float gw = 0.f;
  // incremental Hessian + sweep solve: nv <= 30 and no tendon-limit row in this solve (a
  // model with limited tendons -- the reach scenes -- takes it whenever none is active)
  bool limt = false;
  if (c.nlimt > 0) {
    const int* meta = (const int*)c.f(c.L.efc_meta);
    bool any = false;
    for (int r = LANE; r < nefc; r += DX_WAVE) any |= (meta[r] & 15) == DXR_LIMT;
    limt = __any(any);
  }
  const bool inc = DX_SWEEP && nv <= 30 && !limt;
  // Newton with nv <= 30: M's rows in registers for the solve's products
  const bool mreg = nv <= 30 && c.solver == 2;
  float mr[30];
  if (mreg) mrow_load(c.f(c.L.M), nv, mr);
  float cw = mreg ? eval_cost<true>(c, qacc, Ma, &gw, mr) : eval_cost(c, qacc, Ma, &gw);
  // c.solver is a compile-time constant in a scene specialization (DX_DIMS), so a Newton
  // kernel carries no CG / PGS code
  if (c.solver == 0) {  // the dual solver starts from the warm start's forces
    stage_count(c, CNT_SOLVE);
    stage_count(c, CNT_NEFC, nefc);
    solve_pgs(c, scale, tol);
    return;
  }
  jac_vec(c, a0, jvs);
  for (int r = LANE; r < nefc; r += DX_WAVE) jvs[r] -= aref[r];
  SYNC();
  float cs = rows_cost(c, jvs, 0.f);
  float cost = cw, gauss = gw;
  if (!(cw < cs)) {
    gauss = 0.f;
    for (int i = LANE; i < nv; i += DX_WAVE) { qacc[i] = a0[i]; Ma[i] = qs[i]; }
    for (int r = LANE; r < nefc; r += DX_WAVE) jar[r] = jvs[r];
    SYNC();
    cost = cs;
  }
  int it = 0;
  stage_mark(c, ST_NEWTON_EVAL);
  stage_count(c, CNT_SOLVE);
  stage_count(c, CNT_NEFC, nefc);
  if (c.solver == 1) {
    if (DX_SWEEP && nv <= 30 && nefc <= 2 * DX_WAVE) solve_cg_reg(c, scale, tol);
    else solve_cg(c, scale, tol);
    return;
  }
  float wo[DX_NCH][5] = {};
  for (; it < c.iterations; it++) {
    stage_count(c, CNT_NEWTON_IT);
    jac_t_force(c, grad);  // grad <- J^T f
    float gn = 0;
    for (int i = LANE; i < nv; i += DX_WAVE) {
      grad[i] = Ma[i] - qs[i] - grad[i];
      gn += grad[i] * grad[i];
    }
    gn = sqrtf(wave_sum(gn)) * scale;
    stage_mark(c, ST_NEWTON_GRAD);
    if (gn < tol) break;
    float* H = c.f(c.L.H);
    if (inc) {
      const float hd = build_hessian_inc(c, it == 0, wo);
      stage_mark(c, ST_NEWTON_HESS);
      for (int i = LANE; i < nv; i += DX_WAVE) dir[i] = -grad[i];
      SYNC();
      mfma_sweep_solve30(H, nv, hd, dir);
    } else {
      build_hessian(c);
      stage_mark(c, ST_NEWTON_HESS);
      for (int i = LANE; i < nv; i += DX_WAVE) dir[i] = -grad[i];
      SYNC();
      chol_solve(H, nv, dir, H);
    }
    stage_mark(c, ST_NEWTON_CHOL);
    int changed = 0;
    float nc = 0.f, gnew = 0.f;
    float alpha = inc    ? line_search<true, false, true>(c, qacc, Ma, dir, &changed, nullptr, grad, gauss, &nc, &gnew, mr)
                  : mreg ? line_search<false, false, true>(c, qacc, Ma, dir, &changed, nullptr, nullptr, 0.f, nullptr,
                                                           nullptr, mr)
                         : line_search(c, qacc, Ma, dir, &changed);
    stage_mark(c, ST_NEWTON_LS);
    // qacc += alpha dir; M qacc and J qacc - aref follow by linearity from the line
    // search's M dir (v4) and J dir (efc_jv): no products recomputed (the Newton-mode
    // search wrote the new residuals itself)
    const float* Mdir = c.f(c.L.v4);
    const float* jvd = c.f(c.L.efc_jv);
    for (int i = LANE; i < nv; i += DX_WAVE) {
      qacc[i] += alpha * dir[i];
      Ma[i] += alpha * Mdir[i];
    }
    if (!inc)
      for (int r = LANE; r < nefc; r += DX_WAVE) jar[r] += alpha * jvd[r];
    SYNC();
    // Converged when (a) the full Newton step kept every row in its cost zone: the
    // cost is quadratic on that zone set, so the step landed on its exact minimiser
    // (decided before the cost evaluation, which this exit does not need); or (b) the
    // improvement is below the tolerance or at fp32 noise level of the cost.
    if (changed == 0 && fabsf(alpha - 1.0f) < 1e-3f) {
      it++;
      break;
    }
    if (!inc) nc = total_cost(c, qacc, Ma);
    gauss = gnew;
    stage_mark(c, ST_NEWTON_EVAL);
    float impr = scale * (cost - nc);
    float prev = cost;
    cost = nc;
    if (impr < tol || (prev - nc) <= 1e-9f * fabsf(prev)) {
      it++;
      break;
    }
  }
  if (LANE == 0) c.I[I_NITER] = it;
  SYNC();
}

// ------------------------------------------------------------------------ //
// forward + Euler
// ------------------------------------------------------------------------ //

template <class Ctx>
__device__ __forceinline__ void forward(const Ctx& c, const float* xfrc) {
  const DevModel& m = c.mdl();
  int nv = c.nv;
  // Stage order (LDS phases, see dx_api.hip layout): kinematics/com/crb and the
  // velocity stage use the com temporaries; the smooth solve reuses them for its
  // transpose; collision reuses them for candidates + hull staging; the constraint
  // rows and contact jacobians overwrite those; the Newton Hessian overwrites the
  // kinematic block.  Collision does not depend on velocities, so this order gives
  // the same result as MuJoCo's mj_fwdPosition -> mj_fwdVelocity.
  TenPre tp;
  load_ten_pre(c, tp);
  kin_com(c);
  stage_mark(c, ST_KIN);
  tendon_lengths(c, tp);
  crb_mass(c);
  stage_mark(c, ST_CRB);
  velocity_stage(c, xfrc);
  stage_mark(c, ST_VEL);
  // qacc_smooth = M^-1 qfrc_smooth (Cholesky)
  float* H = c.f(c.L.tsm);
  const float* M = c.f(c.L.M);
  float* a0 = c.f(c.L.qacc_smooth);
  const float* qs = c.f(c.L.qfrc_smooth);
  for (int i = LANE; i < nv; i += DX_WAVE) a0[i] = qs[i];
  SYNC();
  m_solve(c, M, DiagAdd{0.f, 0.f}, a0, H);
  stage_mark(c, ST_SMOOTH);
  collision(c, 0, -1, -1);
  if (c.I[I_DEFER]) return;  // the pool is full: the overflow tier redoes this physics step
  make_constraint(c);
  stage_mark(c, ST_CON);
  solve(c);
  // qfrc_constraint = J^T f at the solution
  float* qc = c.f(c.L.qfrc_con);
  if (c.I[I_NEFC] > 0) {
    jac_t_force(c, qc);
  } else {
    for (int i = LANE; i < nv; i += DX_WAVE) qc[i] = 0;
    SYNC();
  }
  stage_mark(c, ST_QFRC);
}

template <class Ctx>
__device__ __forceinline__ void euler(const Ctx& c, float* time) {
  const DevModel& m = c.mdl();
  int nv = c.nv;
  float h = m.timestep;
  float* qacc = c.f(c.L.qacc);
  float* qvel = c.f(c.L.qvel);
  float* qpos = c.f(c.L.qpos);
  float* acc = c.f(c.L.v1);
  // joint tables before the barriers (njnt <= nv <= 64: one joint per lane)
  const int j0 = min(LANE, c.njnt - 1);
  const int jqa = m.jnt_qposadr[j0], jda = m.jnt_dofadr[j0], jty = m.jnt_type[j0];
  const DiagAdd dd = c.any_damping ? diag_add(m.dof_damping, h, nv) : DiagAdd{0.f, 0.f};
  if (c.any_damping) {
    float* H = c.f(c.L.H);
    const float* M = c.f(c.L.M);
    for (int i = LANE; i < nv; i += DX_WAVE) acc[i] = c.f(c.L.qfrc_smooth)[i] + c.f(c.L.qfrc_con)[i];
    SYNC();
    m_solve(c, M, dd, acc, H);
  } else {
    for (int i = LANE; i < nv; i += DX_WAVE) acc[i] = qacc[i];
    SYNC();
  }
  for (int i = LANE; i < nv; i += DX_WAVE) qvel[i] += h * acc[i];
  SYNC();
  if (LANE < c.njnt) {
    const int qa = jqa, da = jda;
    if (jty == DXJ_FREE) {
      for (int k = 0; k < 3; k++) qpos[qa + k] += h * qvel[da + k];
      float* q = qpos + qa + 3;
      const float* w = qvel + da + 3;
      float wn = norm3(w);
      if (wn > 1e-20f) {
        float ang = h * wn, s, co;
        sincosf(0.5f * ang, &s, &co);
        float dq[4] = {co, w[0] / wn * s, w[1] / wn * s, w[2] / wn * s};
        quatmul(q, q, dq);
      }
      quatnorm(q);
    } else {
      qpos[qa] += h * qvel[da];
    }
  }
  if (LANE == 0) {
    *time += h;
    c.I[I_NSTEP] += 1;
  }
  SYNC();
  stage_mark(c, ST_EULER);
}

// observation pass at the new state: kinematics, com, velocities, sites, watch contact
template <class Ctx>
__device__ __forceinline__ void observe(const Ctx& c, const DevBatch& B, int env) {
  const DevModel& m = c.mdl();
  kin_com(c);
  // cvel (no forces)
  float* qvel = c.f(c.L.qvel);
  float* cdof = c.f(c.L.cdof);
  float* cvel = c.f(c.L.cvel);
  {  // lane = body: cvel as a sum over the body's dof chain (see velocity_stage)
    const int b = LANE;
    if (b < c.nbody) {
      float cv[6] = {0, 0, 0, 0, 0, 0};
      for (uint64_t mask = b >= 1 ? m.body_chain[b] : 0ull; mask; mask &= mask - 1) {
        const int e = __ffsll((long long)mask) - 1;
        const float q = qvel[e];
#pragma unroll
        for (int x = 0; x < 6; x++) cv[x] += cdof[6 * e + x] * q;
      }
#pragma unroll
      for (int x = 0; x < 6; x++) cvel[6 * b + x] = cv[x];
    }
  }
  SYNC();
  float* xpos = c.f(c.L.xpos);
  float* xmat = c.f(c.L.xmat);
  float* rcom = c.f(c.L.rcom);
  for (int s = LANE; s < c.nsite; s += DX_WAVE) {
    int b = m.site_bodyid[s];
    float t[3];
    matvec3(t, xmat + 9 * b, m.site_pos + 3 * s);
    float p[3] = {xpos[3 * b] + t[0], xpos[3 * b + 1] + t[1], xpos[3 * b + 2] + t[2]};
    float* out = B.site_xpos + ((size_t)env * c.nsite + s) * 3;
    out[0] = p[0]; out[1] = p[1]; out[2] = p[2];
    const float* cv = cvel + 6 * b;
    const float* rc = rcom + 3 * m.body_rootidx[b];
    float off[3] = {p[0] - rc[0], p[1] - rc[1], p[2] - rc[2]};
    float wx[3];
    cross3(wx, cv, off);
    float* vo = B.site_vel + ((size_t)env * c.nsite + s) * 6;
    vo[0] = cv[3] + wx[0]; vo[1] = cv[4] + wx[1]; vo[2] = cv[5] + wx[2];
    vo[3] = cv[0]; vo[4] = cv[1]; vo[5] = cv[2];
  }
  // body poses out (when requested) before the watch pass reuses the com-temporary LDS block
  if (B.out_bodies) {
    const float* xq = c.f(c.L.xquat);
    for (int k = LANE; k < 3 * c.nbody; k += DX_WAVE) B.xpos[(size_t)env * 3 * c.nbody + k] = xpos[k];
    for (int k = LANE; k < 4 * c.nbody; k += DX_WAVE) B.xquat[(size_t)env * 4 * c.nbody + k] = xq[k];
  }
  SYNC();
  if (B.watch_geom >= 0 && B.watch) {
    collision(c, 1, B.watch_geom, B.watch_body, B.watch_pairs, B.watch_npairs);
    int n = c.I[I_NCON];
    const float* con = c.f(c.L.con);
    int hit = 0;
    for (int k = LANE; k < n; k += DX_WAVE) hit |= con[DX_CON_STRIDE * k + 12] <= 1e-8f;
    hit = __any(hit);
    if (LANE == 0) B.watch[env] = hit;
  }
}

// ------------------------------------------------------------------------ //
// reach: fingertip goals and collision-free joint angles (mode 2 pass)
// ------------------------------------------------------------------------ //
// Fingertip sites of the current kinematics: lane t < 3 * ntips holds coordinate
// t % 3 of tip t / 3 (site_xpos of dexterous_hand.py:286-291).
template <class Ctx>
__device__ __forceinline__ float tip_coord(const Ctx& c, const TaskParams& P) {
  const DevModel& m = c.mdl();
  float gc = 0;
  if (LANE < 3 * P.ntips) {
    int t = LANE / 3, e = LANE - 3 * t;
    int sid = P.tip_sites[t];
    int b = m.site_bodyid[sid];
    const float* xp = c.f(c.L.xpos) + 3 * b;
    const float* xm = c.f(c.L.xmat) + 9 * b;
    const DXG float* sp = m.site_pos + 3 * sid;
    gc = xp[e] + xm[3 * e] * sp[0] + xm[3 * e + 1] * sp[1] + xm[3 * e + 2] * sp[2];
  }
  return gc;
}
// Any contact with dist <= 1e-8 at the current kinematics (has_self_collision,
// utils/mujoco_collisions.py:95-127; in the reach scenes every contact pair is
// hand-hand because the ground is disabled, reach.py:131-132).
template <class Ctx>
__device__ __forceinline__ bool contact_now(const Ctx& c) {
  collision(c, 0, -1, -1);
  int n = c.I[I_NCON];
  const float* con = c.f(c.L.con);
  int hit = 0;
  for (int k = LANE; k < n; k += DX_WAVE) hit |= con[DX_CON_STRIDE * k + 12] <= 1e-8f;
  return __any(hit) != 0;
}

// numpy RandomState draws for one env, by the whole wave ([3P] numpy legacy MT19937:
// mt19937_gen, legacy_double, legacy_gauss).  The env's 624-word state block is copied
// to LDS scratch (the collision candidate area, free before a pass), outputs pos.. are
// tempered in parallel, and a block that runs out is twisted in place in LDS: chunks
// of 64 in index order, each chunk's loads before its stores, which is the serial
// loop's dependency order (new[k] needs new[k - 227] for k >= 227, new[0] for k = 623).
// The block goes back to HBM only when the draws really consumed past it.
__device__ __forceinline__ void mtw_twist(uint32_t* sm) {
  for (int base = 0; base < 624; base += DX_WAVE) {
    const int k = base + LANE;
    uint32_t a = 0, b = 0, c = 0;
    if (k < 624) { a = sm[k]; b = sm[(k + 1) % 624]; c = sm[(k + 397) % 624]; }
    SYNC();
    if (k < 624) {
      const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
      sm[k] = c ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
    SYNC();
  }
}
struct MtWave {
  uint32_t* g;   // the env's HBM block (DX_MTW_WORDS)
  uint32_t* sm;  // 624 words of LDS
  int pos;       // read position in the current block (uniform)
  bool twisted;  // LDS holds the next block
};
__device__ __forceinline__ MtWave mtw_begin(uint32_t* g, uint32_t* sm) {
  MtWave w;
  w.g = g;
  w.sm = sm;
  // this wave may have rewritten the block earlier in the launch: invalidate the vector
  // L1 so the reloads see those stores
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  for (int k = LANE; k < 624; k += DX_WAVE) sm[k] = g[k];
  w.pos = (int)g[624];
  w.twisted = false;
  SYNC();
  return w;
}
// Outputs [pos, pos + n) of the stream, lane j gets outputs pos + stride*j + t, t < cnt
// (cnt <= 4, n = stride * 64 at most 624); advances pos by `used` (<= n) afterwards
// through mtw_consume.
__device__ __forceinline__ void mtw_fetch(MtWave& w, int stride, int cnt, uint32_t* out) {
  const int n = stride * DX_WAVE;
#pragma unroll
  for (int t = 0; t < 4; t++) {
    const int q = w.pos + stride * LANE + t;
    out[t] = (t < cnt && q < 624) ? dx_mt_temper(w.sm[q]) : 0u;
  }
  if (w.pos + n > 624) {  // part of the batch lies in the next block
    SYNC();
    mtw_twist(w.sm);
#pragma unroll
    for (int t = 0; t < 4; t++) {
      const int q = w.pos + stride * LANE + t;
      if (t < cnt && q >= 624) out[t] = dx_mt_temper(w.sm[q - 624]);
    }
    w.twisted = true;
  }
}
__device__ __forceinline__ void mtw_consume(MtWave& w, int used) {
  if (w.twisted && w.pos + used >= 624) {
    w.pos = w.pos + used - 624;
    for (int k = LANE; k < 624; k += DX_WAVE) w.g[k] = w.sm[k];
  } else if (w.twisted) {  // speculative twist: the stream is still in the old block
    for (int k = LANE; k < 624; k += DX_WAVE) w.sm[k] = w.g[k];
    w.pos += used;
  } else {
    w.pos += used;
  }
  w.twisted = false;
  if (LANE == 0) w.g[624] = (uint32_t)w.pos;
  SYNC();
}
__device__ __forceinline__ double mt_to_double(uint32_t a, uint32_t b) {
  return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) / 9007199254740992.0;
}
// RandomState.uniform(lo, hi) for lanes < n: lo + (hi - lo) * random_sample()
__device__ __forceinline__ double mtw_uniform(MtWave& w, int n, double lo, double hi) {
  uint32_t o[4];
  mtw_fetch(w, 2, 2, o);
  const double u = mt_to_double(o[0], o[1]);
  mtw_consume(w, 2 * n);
  return __dadd_rn(lo, __dmul_rn(hi - lo, u));
}
// RandomState.normal(loc, scale) for lanes < n (legacy_gauss: polar pairs, the second
// value of a pair cached in the state for the next call).  Candidate pairs come 64 at
// a time (lane j: outputs 4j..4j+3); accepted ones are ranked by a ballot.
__device__ __forceinline__ double mtw_normal(MtWave& w, int n, double loc, double scale, double* pairs) {
  int has = (int)w.g[625];
  double cached;
  {
    const uint64_t lo32 = w.g[626], hi32 = w.g[627];
    cached = __longlong_as_double((long long)(lo32 | (hi32 << 32)));
  }
  const int need = n - has;          // gaussians to draw from pairs
  const int npairs = (need + 1) / 2;
  int got = 0;
  while (got < npairs) {
    uint32_t o[4];
    mtw_fetch(w, 4, 4, o);
    const double x1 = 2.0 * mt_to_double(o[0], o[1]) - 1.0;
    const double x2 = 2.0 * mt_to_double(o[2], o[3]) - 1.0;
    const double r2 = __dadd_rn(__dmul_rn(x1, x1), __dmul_rn(x2, x2));
    const bool acc = r2 < 1.0 && r2 != 0.0;
    const uint64_t m = __ballot(acc);
    const int rank = got + __popcll(m & ((1ull << LANE) - 1ull));
    if (acc && rank < npairs) {
      const double f = sqrt(-2.0 * log(r2) / r2);
      pairs[2 * rank] = __dmul_rn(f, x2);      // returned first
      pairs[2 * rank + 1] = __dmul_rn(f, x1);  // cached for the next call
    }
    const int take = min(npairs - got, __popcll(m));
    int used = 4 * DX_WAVE;  // the whole batch unless the last needed pair is in it
    if (take == npairs - got) {
      // lane index of the take-th accepted candidate
      uint64_t mm = m;
      for (int t = 1; t < take; t++) mm &= mm - 1;
      used = 4 * (__ffsll((long long)mm) - 1 + 1);
    }
    got += take;
    mtw_consume(w, used);
  }
  SYNC();
  const int i = LANE;
  double g = 0.0;
  if (i < n) g = (has && i == 0) ? cached : pairs[i - has];
  // state: a leftover second value of the last pair stays cached
  if (LANE == 0 && n > 0) {  // the cached value (if any) was used; an odd count leaves one
    const bool odd = (need & 1) != 0;
    const uint64_t bits = (uint64_t)__double_as_longlong(odd ? pairs[need] : 0.0);
    w.g[625] = odd ? 1u : 0u;
    w.g[626] = (uint32_t)bits;
    w.g[627] = (uint32_t)(bits >> 32);
  }
  SYNC();
  return __dadd_rn(loc, __dmul_rn(scale, g));
}

// FingertipCartesianPosition.next_goal (fingertip_position.py:72-125) and
// DexterousHand.sample_collision_free_joint_angles (dexterous_hand.py:144-168) for
// one environment, with the reference's side effects on the physics state: after a
// goal draw qpos and ctrl are restored, qvel / warm start keep the last rollout's
// values, time advances by the accepted rollout (a rejected one restores it).
// WT: fused into the queued step kernel (fused_reach_prep), where the task state this
// writes is read by the env's last task, which may run on another XCD: write-through.
template <bool WT = false, class Ctx>
__device__ __forceinline__ void reach_prep(const Ctx& c, const DevBatch& B, int env, float& time) {
  using W = TaskStore<WT>;
  const TaskParams& P = *B.tp;
  const TaskState& T = *B.ts;
  float* qpos = c.f(c.L.qpos);
  float* ctrl = c.f(c.L.ctrl);
  float* ws = c.f(c.L.v5);
  const int nq = c.nq, nu = c.nu;
  const int need = T.need[env];
  const int ep = T.episode[env];
  const float* ref = P.tdata;
  const float* lo = ref + nq;
  const float* hi = lo + nq;
  const float* p2c = hi + nq;
  // numpy-compatible draws (P.tdata_f64): the env's RandomState block and the fp64
  // constants after the fp32 tables, lane = joint
  const bool npy = P.tdata_f64 && T.mt_reach;
  const float* f64 = p2c + (size_t)nu * nq;  // raw bits, two words per double (4-byte aligned)
  auto ld64 = [&](int i) -> double {
    const uint64_t lo32 = (uint32_t)__float_as_int(f64[2 * i]), hi32 = (uint32_t)__float_as_int(f64[2 * i + 1]);
    return __longlong_as_double((long long)(lo32 | (hi32 << 32)));
  };
  // (the fp64 constants are loaded at each draw: kept live across the physics rollouts
  // they would push this kernel's registers into scratch)
  const int jl = min(LANE, nq - 1);
  uint32_t* mt_block = npy ? T.mt_reach + (size_t)env * DX_MTW_WORDS : nullptr;
  uint32_t* mt_sm = (uint32_t*)c.f(c.L.cand);  // free before each collision pass
  double* mt_pairs = (double*)c.f(c.L.cand + 624);
  const float q_init = LANE < nq ? qpos[LANE] : 0.f;
  const float c_init = LANE < nu ? ctrl[LANE] : 0.f;
  if (need & 1) {
    const int g = T.goalnum[env];
    float gc = 0;
    bool ok = false;
    int fails = 0;
    for (int att = 0;; att++) {
      // max_rejection_samples draws without a collision-free goal: the reference raises
      // GoalInitializationError (fingertip_position.py:112-117) and GoalEnvironment
      // retries the reset / step (environment.py:14-34) from the continuing RandomState.
      // A retried step re-runs next_goal on the state the failed call restored (the loop
      // below just goes on); a retried reset first resets the physics (mj_resetData)
      if (att > 0 && att % P.max_reject == 0) {
        if (++fails >= DX_GOAL_RETRIES) break;  // bounded here (the reference loops forever)
        if (need & 2) {
          for (int i = LANE; i < c.nv; i += DX_WAVE) { c.f(c.L.qvel)[i] = 0.f; ws[i] = 0.f; }
          time = 0.f;
          if (LANE == 0) c.I[I_NSTEP] = 0;
          SYNC();
        }
      }
      const int a = att;
      // qpos_desired ~ N(midrange, scale * range), clipped to the joint range
      if (npy) {
        MtWave w = mtw_begin(mt_block, mt_sm);
        const double q = mtw_normal(w, nq, ld64(jl), ld64(nq + jl), mt_pairs);
        if (LANE < nq) qpos[LANE] = (float)fmin(ld64(3 * nq + jl), fmax(ld64(2 * nq + jl), q));
      } else if (LANE < nq) {
        const int draw = (int)(0x100000u + (((uint32_t)(g & 4095) * 128u + (uint32_t)(a & 127)) * 64u + LANE) * 2u +
                               ((uint32_t)a >> 7) * 0x4000000u);
        float u1 = dx_urand(P.seed, P.env0 + env, ep, draw), u2 = dx_urand(P.seed, P.env0 + env, ep, draw + 1);
        float z = sqrtf(-2.0f * logf(fmaxf(u1, 1e-12f))) * cosf(6.283185307179586f * u2);
        float l = lo[LANE], h = hi[LANE];
        qpos[LANE] = fminf(h, fmaxf(l, ref[LANE] + P.goal_scale * (h - l) * z));
      }
      SYNC();
      // joint_positions_to_control (shadow_hand_e.py:109-119; identity for Adroit)
      if (LANE < nu) {
        float sacc = 0;
        for (int j = 0; j < nq; j++) sacc += p2c[LANE * nq + j] * qpos[j];
        ctrl[LANE] = sacc;
      }
      SYNC();
      const float t0 = time;
      const int n0 = c.I[I_NSTEP];
      for (int s = 0; s < 2; s++) {  // JointStaticIsolator: two physics steps
        forward(c, B.xfrc);
        for (int i = LANE; i < c.nv; i += DX_WAVE) ws[i] = c.f(c.L.qacc)[i];
        SYNC();
        euler(c, &time);
      }
      kinematics(c);
      gc = tip_coord(c, P);
      // fingertip_position.py:99-103: the accepted goal's joints are the state after
      // the two steps (kept as FingertipCartesianPosition.qpos; the last draw if none)
      if (T.goal_qpos && LANE < nq) W::st(T.goal_qpos, (size_t)env * nq + LANE, qpos[LANE]);
      if (!contact_now(c)) { ok = true; break; }
      time = t0;
      SYNC();
      if (LANE == 0) c.I[I_NSTEP] = n0;
    }
    if (LANE < 3 * P.ntips) W::st(T.goal, (size_t)env * P.goal_dim + LANE, gc);
    if (LANE == 0) {
      W::st(T.goalnum, env, g + 1);
      W::st(T.goalfail, env, T.goalfail[env] + fails + (ok ? 0 : 1));  // GoalInitializationErrors the reference raised (and retried)
      // GoalTask.initialize_episode / before_step bookkeeping (task.py:137-165)
      W::st(T.counter, env, 0);
      W::st(T.exceeded, env, 0);
      W::st(T.registered, env, 0);
      W::st(T.solve_start, env, time);
      W::st(T.solve_n, env, c.I[I_NSTEP]);  // the fp64 start (task_post): the goal's physics step
    }
    if (LANE < nq) qpos[LANE] = q_init;
    if (LANE < nu) ctrl[LANE] = c_init;
    SYNC();
  }
  if (need & 2) {
    // uniform within range_fraction * range, coupled joints equalised, until no contact
    for (int a = 0; a < 1000; a++) {
      if (npy) {
        MtWave w = mtw_begin(mt_block, mt_sm);
        const double q = mtw_uniform(w, nq, ld64(4 * nq + jl), ld64(5 * nq + jl));
        if (LANE < nq) qpos[LANE] = (float)q;
      } else if (LANE < nq) {
        float u = dx_urand(P.seed, P.env0 + env, ep, 0x200000 + a * 64 + LANE);
        float l = P.range_frac * lo[LANE], h = P.range_frac * hi[LANE];
        qpos[LANE] = l + (h - l) * u;
      }
      SYNC();
      if (LANE < P.ncoupled) qpos[P.coupled[LANE][0]] = qpos[P.coupled[LANE][1]];
      SYNC();
      kinematics(c);
      if (!contact_now(c)) break;
    }
  }
  if (LANE == 0) W::st(T.need, env, 0);
  SYNC();
}

// ------------------------------------------------------------------------ //
// kernels
// ------------------------------------------------------------------------ //
// Per-env pieces shared by the launch-per-env kernel and the substep queue.
// env_begin: zero the env's LDS block, load its state; returns its time.
// rec: the env's hand-off record (substeps after the first of a queued step), or null
// for the batch arrays.
template <class Ctx>
__device__ __forceinline__ float env_begin(Ctx& c, const DevBatch& B, int env, const float* rec = nullptr,
                                           bool resume = false) {
  const Lds& L = c.L;
  float* smem = c.S;
  // Zero the whole per-env LDS block: the Cholesky solve reads a few words past its
  // packed triangles (padding lanes/columns, multiplied by exact zeros), and those
  // must be finite rather than whatever an earlier workgroup left behind.
#ifndef DX_SKIP_LDS_ZERO  // (defined only by the test that shows why this is needed)
  for (int k = 4 * LANE; k < L.total; k += 4 * DX_WAVE)  // L.total is a multiple of 4
    *(float4*)(smem + k) = make_float4(0.f, 0.f, 0.f, 0.f);
#endif
  SYNC();
  int* I = c.I;
  if (c.stage_acc && LANE == 0) *(unsigned long long*)(I + 10) = __builtin_amdgcn_s_memtime();
  float* qpos = c.f(L.qpos);
  float* qvel = c.f(L.qvel);
  float* ctrl = c.f(L.ctrl);
  float* ws = c.f(L.v5);
  float time;
  if (rec) {
    for (int i = LANE; i < c.nq; i += DX_WAVE) qpos[i] = rec[i];
    for (int i = LANE; i < c.nv; i += DX_WAVE) {
      qvel[i] = rec[c.nq + i];
      ws[i] = rec[c.nq + c.nv + i];
    }
    time = rec[c.nq + 2 * c.nv];
    if (LANE == 0) {
      I[I_NSTEP] = __float_as_int(rec[c.nq + 2 * c.nv + 2]);
      I[I_FLAGS] = __float_as_int(rec[c.nq + 2 * c.nv + 3]);
    }
  } else {
    for (int i = LANE; i < c.nq; i += DX_WAVE) qpos[i] = B.qpos[(size_t)env * c.nq + i];
    for (int i = LANE; i < c.nv; i += DX_WAVE) {
      qvel[i] = B.qvel[(size_t)env * c.nv + i];
      ws[i] = B.qacc_ws[(size_t)env * c.nv + i];
    }
    time = B.time[env];
    if (LANE == 0) {
      I[I_NSTEP] = B.nstep ? B.nstep[env] : 0;
      // (the overflow tier resuming a deferred control step: its earlier physics steps'
      // divergence flag, which health_check stored write-through)
      I[I_FLAGS] = resume && B.bad ? (B.bad[env] & 1) : 0;
    }
  }
  for (int i = LANE; i < c.nu; i += DX_WAVE) ctrl[i] = B.ctrl[(size_t)env * c.nu + i];
  if (LANE < I_NINT) I[LANE] = 0;
  SYNC();
  return time;
}

template <class Ctx>
__device__ __forceinline__ void env_store_state(const Ctx& c, const DevBatch& B, int env, float time) {
  const float* qpos = c.f(c.L.qpos);
  const float* qvel = c.f(c.L.qvel);
  const float* ws = c.f(c.L.v5);
  for (int i = LANE; i < c.nq; i += DX_WAVE) B.qpos[(size_t)env * c.nq + i] = qpos[i];
  for (int i = LANE; i < c.nv; i += DX_WAVE) {
    B.qvel[(size_t)env * c.nv + i] = qvel[i];
    B.qacc_ws[(size_t)env * c.nv + i] = ws[i];
  }
  if (LANE == 0) {
    B.time[env] = time;
    if (B.nstep) B.nstep[env] = c.I[I_NSTEP];
  }
}

// The hand-off record (DevBatch::hand) of a task whose env has substeps left: lane t
// gathers words 4t .. 4t + 3 from LDS and writes them with one 16-byte sc1 store.
template <class Ctx>
__device__ __forceinline__ void env_store_hand(const Ctx& c, float* rec, int stride, float time, unsigned cost) {
  const float* qpos = c.f(c.L.qpos);
  const float* qvel = c.f(c.L.qvel);
  const float* ws = c.f(c.L.v5);
  const int nw = c.nq + 2 * c.nv + 4;
  time = rl(time, 0);  // euler advances time in lane 0 only
  const int nstep = c.I[I_NSTEP], flags = c.I[I_FLAGS];
  for (int t = LANE; 4 * t < nw; t += DX_WAVE) {
    float w[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int m = 4 * t + u, k = m - (c.nq + 2 * c.nv);
      w[u] = m < c.nq ? qpos[m]
           : m < c.nq + c.nv ? qvel[m - c.nq]
           : m < c.nq + 2 * c.nv ? ws[m - c.nq - c.nv]
           : k == 0 ? time : k == 1 ? __uint_as_float(cost) : k == 2 ? __int_as_float(nstep) : __int_as_float(flags);
    }
    st_sc1_f4(rec, 4 * stride, 16 * t, make_float4(w[0], w[1], w[2], w[3]));
  }
}

// Torque sensors (dx_sensor.hip), when enabled: the state the sensors of mj_step2
// read -- pre-integration qpos / qvel, the solved qacc -- and every contact's bodies,
// point and world-frame force on body 2 (the contact-frame forces jac_t_force left in
// cw, decoded from the pyramid rows, rotated by the contact frame).
template <class Ctx>
__device__ __forceinline__ void sensor_stash(const Ctx& c, const DevBatch& B, int env) {
  const DevModel& m = c.mdl();
  const int nq = c.nq, nv = c.nv;
  float* o = B.sen_stash + (size_t)env * (nq + 2 * nv + 1 + 8 * DX_NCON_HI);
  for (int i = LANE; i < nq; i += DX_WAVE) o[i] = c.f(c.L.qpos)[i];
  for (int i = LANE; i < nv; i += DX_WAVE) {
    o[nq + i] = c.f(c.L.qvel)[i];
    o[nq + nv + i] = c.f(c.L.qacc)[i];
  }
  const int n = c.I[I_NEFC] > 0 ? c.I[I_NCON] : 0;
  if (LANE == 0) o[nq + 2 * nv] = __int_as_float(n);
  const float* con = c.f(c.L.con);
  const float* cw = c.f(c.L.cw);
  for (int ci = LANE; ci < n; ci += DX_WAVE) {
    const float* r = con + DX_CON_STRIDE * ci;
    const int gp = __float_as_int(r[13]);
    float* q = o + nq + 2 * nv + 1 + 8 * ci;
    q[0] = __int_as_float(m.geom_bodyid[m.gpair_geom[2 * gp]]);
    q[1] = __int_as_float(m.geom_bodyid[m.gpair_geom[2 * gp + 1]]);
    q[2] = r[0]; q[3] = r[1]; q[4] = r[2];
    const float f0 = cw[3 * ci], f1 = cw[3 * ci + 1], f2 = cw[3 * ci + 2];
    for (int k = 0; k < 3; k++) q[5 + k] = r[3 + k] * f0 + r[6 + k] * f1 + r[9 + k] * f2;
  }
}

// After a physics step: the capacity bits of its collision / constraint passes go to
// the batch's always-on health counters (include/dx.h dx_health), and a state that is no
// longer finite -- or an acceleration beyond mjMAXVAL -- is MuJoCo's BADQACC
// ([3P] mj_checkAcc): the env's data is reset (mj_resetData: qpos0, zero velocity, warm
// start, ctrl and time), the env is flagged (B.bad, which the task turns into dm_control's
// divergent-physics step: LAST, reward 0, discount 0) and counted.
template <class Ctx>
__device__ __forceinline__ void health_check(const Ctx& c, const DevBatch& B, int env, float& time, bool reset = true) {
  const DevModel& m = c.mdl();
  int* I = c.I;
  const int ovf = I[I_OVF], nraw = I[I_NRAW];
  const float* qpos = c.f(c.L.qpos);
  const float* qvel = c.f(c.L.qvel);
  const float* qacc = c.f(c.L.qacc);
  bool badl = false;
  for (int i = LANE; i < c.nq; i += DX_WAVE) badl |= !isfinite(qpos[i]);
  for (int i = LANE; i < c.nv; i += DX_WAVE) badl |= !isfinite(qvel[i]) || !(fabsf(qacc[i]) <= DX_MAXVAL);
  const bool bad = __any(badl) != 0;
  if (LANE == 0 && B.health) {
    if (ovf & 1) atomicAdd(B.health + 1, 1u);
    if (ovf & 2) atomicAdd(B.health + 0, 1u);
    if (ovf & 4) atomicAdd(B.health + 2, 1u);
    if (ovf & 8) atomicAdd(B.health + 3, 1u);
    if (bad) atomicAdd(B.health + 4, 1u);
    if (nraw > 16) atomicMax(B.health + 5, (unsigned)nraw);
    if (B.ncon_hist) atomicAdd(B.ncon_hist + min(nraw, DX_NCON_HIST - 1), 1u);
  }
  SYNC();
  if (LANE == 0) { I[I_OVF] = 0; I[I_NRAW] = 0; }
  if (bad && !reset) {  // mj_forward: flagged and counted ([3P] mj_checkAcc runs in mj_step only)
    if (LANE == 0 && B.bad && env >= 0) TaskStore<true>::st(B.bad, env, 1);
  } else if (bad) {
    float* q = c.f(c.L.qpos);
    for (int i = LANE; i < c.nq; i += DX_WAVE) q[i] = m.qpos0[i];
    for (int i = LANE; i < c.nv; i += DX_WAVE) {
      c.f(c.L.qvel)[i] = 0.f;
      c.f(c.L.v5)[i] = 0.f;  // warm start
      c.f(c.L.qacc)[i] = 0.f;
    }
    for (int i = LANE; i < c.nu; i += DX_WAVE) {
      c.f(c.L.ctrl)[i] = 0.f;
      // later substeps (queued tasks, maybe on another XCD) reload it: write-through
      if (env >= 0) TaskStore<true>::st(B.ctrl, (size_t)env * c.nu + i, 0.f);
    }
    time = 0.f;
    if (LANE == 0) {
      c.I[I_NSTEP] = 0;
      c.I[I_FLAGS] |= 1;
      if (B.bad && env >= 0) TaskStore<true>::st(B.bad, env, 1);  // (read after the launch)
    }
  }
  SYNC();
}

// One physics step (mj_step): forward, warm start <- solved qacc, Euler, health check.
template <class Ctx>
__device__ __forceinline__ void env_substep(const Ctx& c, const DevBatch& B, float& time, int env, bool last) {
  forward(c, B.xfrc);
  if (c.I[I_DEFER]) return;  // (the state in LDS is still the one this physics step started from)
  if (last && B.sen_stash) sensor_stash(c, B, env);
  float* ws = c.f(c.L.v5);
  for (int i = LANE; i < c.nv; i += DX_WAVE) ws[i] = c.f(c.L.qacc)[i];
  SYNC();
  euler(c, &time);
  health_check(c, B, env, time);
}

// After the last substep (or a forward): debug record, per-env outputs, the
// observation pass at the new state, and the state itself.
template <class Ctx>
__device__ __forceinline__ void env_finish(const Ctx& c, const DevBatch& B, int env, float time) {
  const DevModel& m = c.mdl();
  const Lds& L = c.L;
  int* I = c.I;
  if (B.dbg_qacc_smooth) {
    for (int i = LANE; i < c.nv; i += DX_WAVE) {
      B.dbg_qacc_smooth[(size_t)env * c.nv + i] = c.f(L.qacc_smooth)[i];
      B.dbg_qfrc_smooth[(size_t)env * c.nv + i] = c.f(L.qfrc_smooth)[i];
    }
    for (int k = LANE; k < c.nv * c.nv; k += DX_WAVE) {
      int i = k / c.nv, j = k % c.nv;
      B.dbg_M[(size_t)env * c.nv * c.nv + k] = c.f(L.M)[i >= j ? ti(i) + j : ti(j) + i];
    }
    int n = I[I_NCON];
    for (int k = LANE; k < DX_NCON_HI * 16; k += DX_WAVE) {
      int ci = k / 16, e = k % 16;
      float v = 0;
      if (ci < n) {
        const float* r = c.f(L.con) + DX_CON_STRIDE * ci;
        if (e < 13) v = r[e];
        else {
          int gp = __float_as_int(r[13]);
          v = e == 13 ? (float)m.gpair_geom[2 * gp] : e == 14 ? (float)m.gpair_geom[2 * gp + 1] : (float)m.gpair_condim[gp];
        }
      }
      B.dbg_con[(size_t)env * DX_NCON_HI * 16 + k] = v;
    }
    if (LANE == 0) { B.dbg_nefc[2 * env] = I[I_NEFC]; B.dbg_nefc[2 * env + 1] = I[I_OVF]; }
  }
  if (LANE == 0) {
    B.ncon[env] = I[I_NCON];
    B.niter[env] = I[I_NITER];
    B.ncand[env] = I[I_NCAND];
  }
  for (int i = LANE; i < c.nv; i += DX_WAVE) B.qacc[(size_t)env * c.nv + i] = c.f(L.qacc)[i];
  SYNC();
  stage_mark(c, ST_IO);
  observe(c, B, env);
  stage_mark(c, ST_OBSERVE);
  env_store_state(c, B, env, time);
}

// The next launch's longest-first order (DevBatch::ohist / okey): the env's cost bucket
// (descending cost) counted, its rank within the bucket kept.  Called once per env and
// launch, when its control step ends (or goes to the overflow tier: the top bucket).
__device__ __forceinline__ void order_key(const DevBatch& B, int env, unsigned cost) {
  if (B.onext && LANE == 0) {
    const unsigned b = 255u - min(cost >> 4, 255u);
    const unsigned r = atomicAdd(B.ohist + 256 * B.opar + b, 1u);
    B.okey[env] = b << DX_OKEY_RANK_BITS | r;  // 24-bit rank: every env of a batch (<= 2^20) in one bucket
  }
}

// A physics step whose contacts overflow the step kernel's pool (I_DEFER) is handed,
// from the state it started from, to the overflow tier: the state goes to the batch
// arrays, the env to the deferral list (substep s; forward-only for a dx_forward), its
// cost to the top bucket of the next launch's longest-first order, and the count of
// deferrals to the health counters.  Nothing of the env is written after this.
// With the mid tier running beside the launch (B.mid, queued mode 0 only) the deferral is
// published while the launch runs: the state goes write-through (sc1) into the env's
// hand-off record, vmcnt drains, and only then is the entry stored (relaxed, agent scope,
// DX_DEFER_VALID set) -- the queue's own hand-off protocol.  `list` is the deferral list:
// B.defer from the step kernel, B.defer2 from the mid tier (the health count of deferrals
// counts the step kernel's only).
template <class Ctx>
__device__ __forceinline__ void env_defer(const Ctx& c, const DevBatch& B, int env, int s, bool fwd, float time,
                                          unsigned* list = nullptr) {
  const bool publish = B.mid && list == nullptr;
  if (!list) list = B.defer;
  const unsigned val = (unsigned)env | ((unsigned)s << DX_DEFER_ENV_BITS) | (fwd ? DX_DEFER_FWD : 0u);
  if (publish) {
    env_store_hand(c, B.hand + (size_t)env * B.hand_stride, B.hand_stride, time, 0u);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    env_store_state(c, B, env, rl(time, 0));
  }
  if (LANE == 0) {
    // the launch that owns the list's entries (list[1]): the mid tier claims only its own
    // launch's (defer_claim), so a mid tier that starts while an earlier launch's step
    // kernel still publishes leaves those entries to that launch's overflow tier
    if (publish) {
      __hip_atomic_store(list + 1, B.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const unsigned k = atomicAdd(list, 1u);
    if (publish)
      __hip_atomic_store(list + 2 + k, val | DX_DEFER_VALID, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else
      list[2 + k] = val;
    if (B.cost) B.cost[env] = 0xffffffffu;
    if (B.health) {
      if (list == B.defer) atomicAdd(B.health + 6, 1u);
      atomicMax(B.health + 5, (unsigned)c.I[I_NRAW]);
    }
  }
  if (!fwd && list == B.defer) order_key(B, env, 0xffffffffu);
}

// Deferral entries beside a mid-tier launch: either consumer -- the mid tier while the
// launch runs, or the overflow tier after it, should the mid tier not have run (a
// profiler or a shared hardware queue serialising the two streams) -- takes an entry by
// compare-and-swap.  Lane 0: 1 taken (*e its value), 2 taken by the other consumer, 0 not
// published yet (or, epoch != 0: published by another launch than `epoch`, list[1] --
// the mid tier runs only its own launch's entries, with its own launch's arguments).
// The claim compares the whole entry, so an entry read before the overflow tier reset the
// list and republished by the next launch is taken only if it is that launch's same entry.
__device__ __forceinline__ int defer_claim(unsigned* list, unsigned i, unsigned* e, unsigned epoch = 0u) {
  unsigned v = __hip_atomic_load(list + 2 + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (epoch && (v & DX_DEFER_VALID)) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (__hip_atomic_load(list + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != epoch) return 0;
  }
  for (;;) {
    if (!(v & DX_DEFER_VALID)) return 0;
    if (v & DX_DEFER_CLAIMED) return 2;
    if (__hip_atomic_compare_exchange_strong(list + 2 + i, &v, v | DX_DEFER_CLAIMED, __ATOMIC_RELAXED,
                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
      *e = v;
      return 1;
    }
  }
}
__device__ __forceinline__ int defer_env(unsigned e) { return (int)(e & ((1u << DX_DEFER_ENV_BITS) - 1u)); }
__device__ __forceinline__ int defer_step(unsigned e) { return (int)((e >> DX_DEFER_ENV_BITS) & 255u); }

// Fused task_pre (DevBatch::fuse) in the env's first physics-step task: before_step /
// initialize_episode by lane 0, then ctrl = the action (zero after a reset), every lane,
// write-through -- the env's later tasks may run on other XCDs.  Returns 1 when the env
// was (re)initialised (FIRST: observed only).  The workgroup fence makes lane 0's batch
// stores (a reset's state) visible to the env_begin that follows.
template <class Ctx>
__device__ __forceinline__ int fused_pre(const Ctx& c, const DevBatch& B, int env) {
  const TaskParams& P = *(const TaskParams*)(const DXG TaskParams*)B.tp;
  const TaskState& S = *(const TaskState*)(const DXG TaskState*)B.ts;
  int skip = 0;
  if (LANE == 0) skip = task_pre<true>(P, S, B, c.mdl().qpos0, env);
  skip = __shfl(skip, 0, 64);
  for (int i = LANE; i < c.nu; i += DX_WAVE) {
    const size_t k = (size_t)env * c.nu + i;
    const float a = skip ? 0.f
                  : B.act_random ? random_action(c.mdl().actuator_ctrlrange, B.act_seed, P.env0 + env, B.act_step, i)
                  : B.action ? B.action[k] : B.ctrl[k];
    TaskStore<true>::st(B.ctrl, k, a);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  return skip;
}

// Fused task_post in the env's last task, after env_finish wrote its outputs: after_step,
// reward, discount, termination and the observation (dx_task.h).
template <class Ctx>
__device__ __forceinline__ void fused_post(const Ctx& c, const DevBatch& B, int env, bool skip) {
  const TaskParams& P = *(const TaskParams*)(const DXG TaskParams*)B.tp;
  const TaskState& S = *(const TaskState*)(const DXG TaskState*)B.ts;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  task_post(P, S, B, env, LANE, skip, (c.I[I_FLAGS] & 1) != 0, c.I[I_NSTEP]);
}

// Fused reach (DevBatch::fuse, a reach scene's specialization): after task_pre, an env
// that requested a goal or initial joints (S.need, set by task_pre) runs the sampling pass
// (reach_prep: goal rollouts, joint sampling) right here, in its first physics-step task,
// instead of in a mode-2 launch of its own; the state it leaves goes through the batch
// arrays and is reloaded into a zeroed LDS block, as the separate pass hands it to the
// step kernel, so the result is the unfused one bit for bit.  Returns the env's time.
template <class Ctx>
__device__ __forceinline__ float fused_reach_prep(Ctx& c, const DevBatch& B, int env, float time) {
  const TaskState& S = *(const TaskState*)(const DXG TaskState*)B.ts;
  // (a reach scene's specialization; the guard keeps another task on a layout-equal
  // scene from reading reach state it does not keep)
  if (((const DXG TaskParams*)B.tp)->kind != DX_KIND_REACH) return time;
  int need = 0;
  if (LANE == 0) need = S.need[env];
  if (!__builtin_amdgcn_readfirstlane(need)) return time;
  const bool defer = c.defer;
  c.defer = false;  // (the sampling pass keeps its pool and cuts it, as mode 2 does)
  reach_prep<true>(c, B, env, time);
  c.defer = defer;
  env_store_state(c, B, env, rl(time, 0));
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  return env_begin(c, B, env);
}

// mode 0: nsub x (forward + Euler), then observe;  mode 1: forward only (+observe)
// mode 2: reach sampling pass (goal rollouts / joint sampling), state out only
template <class SP>
__device__ __forceinline__ void step_body(const DevModel& m, const DevBatch& B, const Lds& Lrt, int nsub, int mode,
                                          bool prep = false) {
  extern __shared__ float smem[];
  if ((int)blockIdx.x >= B.nenv) return;
  // longest-first dispatch: the order kernel sorts envs by their last step's cost
  int env = B.order ? B.order[blockIdx.x] : (int)blockIdx.x;
  const unsigned long long t_start = __builtin_amdgcn_s_memtime();
  if (mode == 2 && !B.ts->need[env]) return;
  CtxT<SP> c(m, Lrt, smem, nullptr, B.stage_acc ? B.stage_acc + (size_t)env * DX_NSTAGE : nullptr);
  c.I = (int*)(smem + c.L.ints);
  c.sep = B.sepcache ? B.sepcache + (size_t)env * DX_SEP_SLOTS : nullptr;
  c.np_wide = B.np_wide;
  c.defer_at = B.defer_at;
  c.defer = !prep && B.defer;  // (the reach sampling pass keeps its pool and cuts it)
  if (prep) {  // reach sampling pass (mode 2): new state only, no outputs
    float time = env_begin(c, B, env);
    reach_prep(c, B, env, time);
    env_store_state(c, B, env, time);
    return;
  }
  // DX_DIVERGED reports this call: cleared here, set by health_check (both write-through)
  if (LANE == 0 && B.bad) TaskStore<true>::st(B.bad, env, 0);
  const bool fuse = B.fuse && mode == 0;
  int skip = fuse ? fused_pre(c, B, env) : (B.skip && B.skip[env]);
  float time = env_begin(c, B, env);
  if constexpr (SP::reach_task)
    if (fuse) time = fused_reach_prep(c, B, env, time);
  const int steps = skip ? 0 : mode == 0 ? nsub : 1;  // a freshly reset env is only observed
  for (int s = 0; s < steps; s++) {
    if (mode == 0) {
      env_substep(c, B, time, env, s == steps - 1);
    } else {
      forward(c, B.xfrc);
      if (!c.I[I_DEFER]) {
        if (B.sen_stash) sensor_stash(c, B, env);
        health_check(c, B, env, time, false);
      }
    }
    if (c.I[I_DEFER]) {
      env_defer(c, B, env, s, mode != 0, time);
      return;
    }
  }
  env_finish(c, B, env, time);
  if (mode == 0) {
    const unsigned cost = (unsigned)min((__builtin_amdgcn_s_memtime() - t_start) >> 10, 0xffffffffull);
    if (LANE == 0 && B.cost) B.cost[env] = cost;
    if (fuse) fused_post(c, B, env, skip);
    order_key(B, env, cost);
  }
}

// Substep queue (mode 0): one task = one physics step of one environment, claimed in
// order from a device counter -- substep s of every env of the queue (longest-first
// within the round) before substep s + 1 of any.  There is one queue per XCD: queue q
// holds the envs at positions q, q + 8, q + 16, ... of the longest-first order, and a
// workgroup claims from its own XCD's queue (HW_REG_XCC_ID), so an env's five tasks
// normally run under one L2 and its hand-offs and separating-direction cache are L2
// hits, not fabric round trips.  When its queue is empty the workgroup takes tasks
// from the next queues.  Placement only decides speed: the hand-off protocol below is
// the cross-XCD one whichever workgroup takes a task.  The env's state moves between its tasks
// through its hand-off record (DevBatch::hand, 3 lines for a Shadow hand) and its
// separating-direction cache, so the wave slots stay
// busy until the last round instead of idling behind the few environments whose
// control step is 2-3x the mean (a whole control step per workgroup left most of
// the second round's slots waiting on them).  Task (s, e) waits for (s - 1, e),
// which was claimed earlier by a running workgroup, so the wait always ends; it is
// bounded anyway (B.qerr records a timeout).  Hand-off (MI355X guide, Guideline 16
// R1): the producer stores the handed-off bytes write-through (sc1), drains vmcnt and
// stores the progress tag relaxed at agent scope (sc1); the consumer polls relaxed,
// then one agent acquire + vmcnt(0) before its plain loads.  With the task logic fused
// (DevBatch::fuse), the env's first task runs task_pre (its writes that later tasks read
// are write-through too) and its last task_post.
__device__ __forceinline__ unsigned qtag(unsigned epoch, int s) { return epoch * 32u + (unsigned)s; }
#define DX_TAG_DEFER 31  // progress tag of an env whose control step went to the overflow tier
#define DX_TAG_DONE 30   // ... whose control step ended in its first task (a fresh reset: observed only)
#define DX_QUEUE_NSUB 29 // longest control step the queue takes (tags 30, 31 are markers)

template <class SP>
__device__ __forceinline__ void step_queue(const DevModel& m, const DevBatch& B, const Lds& Lrt, int nsub) {
  extern __shared__ float smem[];
  CtxT<SP> c(m, Lrt, smem, nullptr, nullptr);
  c.I = (int*)(smem + c.L.ints);
  c.np_wide = B.np_wide;
  c.defer_at = B.defer_at;
  c.defer = B.defer != nullptr;
  const int nqueue = B.nqueue;
  unsigned xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  int q = (int)((xcc & 7u) % (unsigned)nqueue);
  int empty = 0;  // queues found drained, in the order this workgroup visits them
  for (;;) {
    // queue q: order positions q + nqueue * j, j < nq
    const unsigned nq = B.nenv > q ? (unsigned)(B.nenv - q + nqueue - 1) / (unsigned)nqueue : 0u;
    unsigned t = 0;
    if (LANE == 0) t = __hip_atomic_fetch_add(B.qhead + q * DX_QHEAD_STRIDE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    t = __builtin_amdgcn_readfirstlane(t);
    if (t >= nq * (unsigned)nsub) {
      if (++empty >= nqueue) break;
      q = q + 1 == nqueue ? 0 : q + 1;
      continue;
    }
    const int s = (int)(t / nq);
    const int k = q + nqueue * (int)(t - (unsigned)s * nq);
    const int env = B.order ? B.order[k] : k;
    if (s > 0) {
      int abort = 0;
      if (LANE == 0) {
        unsigned n = 0;
        const unsigned long long w0 = B.stage_acc ? __builtin_amdgcn_s_memtime() : 0ull;
        for (;;) {
          const unsigned tag = __hip_atomic_load(B.progress + env, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (tag == qtag(B.epoch, s)) break;
          // an earlier physics step of the env went to the overflow tier, which runs the
          // rest of its control step, or the control step ended in its first task:
          // nothing to do here
          if (tag == qtag(B.epoch, DX_TAG_DEFER) || tag == qtag(B.epoch, DX_TAG_DONE)) { abort = 2; break; }
          __builtin_amdgcn_s_sleep(2);
          // ~seconds without progress (never expected), or another task gave up: the
          // launch is aborted -- no task computes on a state whose predecessor has
          // not been published, and the next dx_sync reports the error
          if (++n > (1u << 25)) {
            __hip_atomic_store(B.qerr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            abort = 1;
            break;
          }
          if ((n & 1023u) == 0 && __hip_atomic_load(B.qerr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
            abort = 1;
            break;
          }
        }
        // (profiling: the cycles this slot waited for the env's previous physics step)
        if (B.stage_acc) stage_add(B.stage_acc + (size_t)env * DX_NSTAGE + CNT_QWAIT, __builtin_amdgcn_s_memtime() - w0);
      }
      if (__builtin_amdgcn_readfirstlane(abort)) continue;  // drain (or deferred / done): later claims end the loop
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const unsigned long long t_start = __builtin_amdgcn_s_memtime();
    c.stage_acc = B.stage_acc ? B.stage_acc + (size_t)env * DX_NSTAGE : nullptr;
    c.sep = B.sepcache ? B.sepcache + (size_t)env * DX_SEP_SLOTS : nullptr;
    float* rec = B.hand + (size_t)env * B.hand_stride;
    // cost so far (shader cycles / 1024), carried in the record between substeps
    const unsigned cost0 = s > 0 ? __float_as_uint(rec[c.nq + 2 * c.nv + 1]) : 0u;
    int skip = 0;
    if (s == 0) {
      // DX_DIVERGED reports this call: cleared here, set by health_check (write-through)
      if (LANE == 0 && B.bad) TaskStore<true>::st(B.bad, env, 0);
      skip = B.fuse ? fused_pre(c, B, env) : (B.skip && B.skip[env]);
    }
    float time = env_begin(c, B, env, s > 0 ? rec : nullptr);
    if constexpr (SP::reach_task)
      if (s == 0 && B.fuse) time = fused_reach_prep(c, B, env, time);
    if (!skip && !(s > 0 && !B.fuse && B.skip && B.skip[env])) env_substep(c, B, time, env, s == nsub - 1);
    if (c.I[I_DEFER]) {
      env_defer(c, B, env, s, false, time);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (LANE == 0) __hip_atomic_store(B.progress + env, qtag(B.epoch, DX_TAG_DEFER), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      continue;
    }
    const bool last = s == nsub - 1 || (skip && B.fuse);  // (a fresh reset is observed right away)
    const unsigned tcost = (unsigned)min((__builtin_amdgcn_s_memtime() - t_start) >> 10, 0xffffffffull);
    const unsigned cost = cost0 + tcost;
    if (last) {
      env_finish(c, B, env, time);
      if (LANE == 0 && B.cost) B.cost[env] = cost;
      if (B.fuse) fused_post(c, B, env, skip);
      // the next launch's longest-first key: this control step's cost, or (DX_ORDER_LAST 1)
      // its last physics step's x nsub, or (2) the mean of the two
      const unsigned lcost = tcost * (unsigned)nsub;
      order_key(B, env, skip || !B.order_last ? cost : B.order_last == 1 ? lcost : (cost >> 1) + (lcost >> 1));
    } else {
      env_store_hand(c, rec, B.hand_stride, time, cost);
    }
    // publish: the bytes the env's next task must read (the hand-off record) were
    // stored write-through (sc1), so a drained vmcnt suffices and no release fence (a
    // write-back of the whole XCD L2) is needed.  The separating-direction cache is
    // stored plainly: a stale entry on another XCD changes no result (narrow_pass).
    // Profiling runs also carry stage_acc across tasks with plain stores: those keep
    // the release.
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (B.stage_acc) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (LANE == 0)
      __hip_atomic_store(B.progress + env, qtag(B.epoch, last && s < nsub - 1 ? DX_TAG_DONE : s + 1), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
  }
  // the mid tier's end-of-launch signal: every deferral of this workgroup was published
  // (its count atomic returned before the entry store) before this count
  if (B.mid && LANE == 0) __hip_atomic_fetch_add(B.qdone, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ------------------------------------------------------------------------ //
// model specializations (build.py writes dx_specs.inc from the shipped scenes)
// ------------------------------------------------------------------------ //
// build.py compiles this file once per specialization with -DDX_SPEC_ONLY=<spec>
// (that translation unit holds only that scene's kernel and its launcher), and once
// without it (generic kernel, dispatch, helper kernels), so the kernels compile in
// parallel.
#if __has_include("dx_specs.inc") && !defined(DX_TIER_HI) && !defined(DX_TIER_MID)
#include "dx_specs.inc"
#endif
#ifndef DX_SPECS
#define DX_SPECS(X)
#endif

#ifndef DX_STEP_WAVES
#define DX_STEP_WAVES 2  // waves per SIMD the VGPR budget is set for (3: <= 168 VGPRs, measured slower)
#endif
// The substep queue (mode 3) is a kernel of its own: the step kernel's code -- every stage
// inlined -- is ~0.4 MB per entry point, and one kernel holding both the queue and the
// one-workgroup-per-env path doubled what the wave slots of a CU fetch into their shared
// instruction cache.
template <class SP>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(DX_STEP_WAVES)))
dx_step_kernel_spec(const DevModel* __restrict__ mp, DevBatch B, Lds L, int nsub, int mode) {
  const DevModel& m = *(const DevModel*)(const DXG DevModel*)mp;
  step_body<SP>(m, B, L, nsub, mode);
}
template <class SP>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(DX_STEP_WAVES)))
dx_step_kernel_queue_spec(const DevModel* __restrict__ mp, DevBatch B, Lds L, int nsub) {
  const DevModel& m = *(const DevModel*)(const DXG DevModel*)mp;
  step_queue<SP>(m, B, L, nsub);
}
// Mode 2 (reach goal rollouts / joint sampling) is its own kernel, so the rarely-run
// sampling code does not share the step kernel's register allocation.
template <class SP>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2)))
dx_prep_kernel_spec(const DevModel* __restrict__ mp, DevBatch B, Lds L) {
  const DevModel& m = *(const DevModel*)(const DXG DevModel*)mp;
  step_body<SP>(m, B, L, 1, 2, true);
}

template <class SP>
static bool spec_matches(const DevModel& d, const Lds& L) {
  if (memcmp(&SP::L, &L, sizeof(Lds)) != 0) return false;
#define DX_X(n) if (SP::n != d.n) return false;
  DX_DIMS(DX_X)
#undef DX_X
  return true;
}

#define DX_SPEC_FNS(SP)                                                                               \
  bool dx_match_##SP(const DevModel& d, const Lds& L);                                                \
  int dx_occ_##SP(size_t lds);                                                                        \
  hipError_t dx_launch_##SP(int grid, size_t lds, hipStream_t stream, const DevModel* m, const DevBatch& B, \
                            const Lds& L, int nsub, int mode);

#if defined(DX_TIER_HI)
// ------------------------------------------------------------------------ //
// overflow tier (build.py compiles this file once more with -DDX_TIER_HI
// -DDX_NCON_MAX=DX_NCON_HI): the physics steps the step kernel deferred (env_defer),
// each run by one workgroup with the DX_NCON_HI pool, from the state it was deferred at
// to the end of the env's control step (or its forward pass), with the step kernel's
// outputs.  Launched behind every step-kernel launch; it exits at once when nothing was
// deferred, which is nearly always (profiles/r3a_ncon_hist.json: 3.4e-6 of env-substeps).
// ------------------------------------------------------------------------ //
static_assert(DX_NCON_MAX == DX_NCON_HI, "the overflow tier is compiled with the DX_NCON_HI pool");
// The same launch also places every env of the next launch's longest-first order
// (DevBatch::ohist / okey, written by the step kernel: order_key) -- each workgroup a
// slice of the envs, from the bucket prefix it computes itself -- and its last workgroup
// zeroes that histogram and the substep-queue heads for the next step-kernel launch.
extern "C" __global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1)))
dx_step_hi_kernel(const DevModel* __restrict__ mp, DevBatch B, Lds L, int nsub) {
  extern __shared__ float smem[];
  const DevModel& m = *(const DevModel*)(const DXG DevModel*)mp;
  // 1. the order: bucket prefix (four buckets per lane), then this workgroup's envs
  if (B.onext && B.order) {
    const unsigned* h = B.ohist + 256 * B.opar;
    unsigned hv[4], sum = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) { hv[k] = h[4 * LANE + k]; sum += hv[k]; }
    const unsigned ex = (unsigned)wave_incl_scan((int)sum) - sum;
    unsigned pre[4];
    pre[0] = ex; pre[1] = ex + hv[0]; pre[2] = pre[1] + hv[1]; pre[3] = pre[2] + hv[2];
    const int per = (B.nenv + (int)gridDim.x - 1) / (int)gridDim.x;
    const int e0 = (int)blockIdx.x * per, e1 = min(B.nenv, e0 + per);
    for (int base = e0; base < e1; base += DX_WAVE) {  // uniform trip count (the shuffles)
      const int e = base + LANE;
      const unsigned key = e < e1 ? B.okey[e] : 0u;
      const int b = (int)(key >> DX_OKEY_RANK_BITS);
      const unsigned p0 = __shfl(pre[0], b >> 2, 64), p1 = __shfl(pre[1], b >> 2, 64);
      const unsigned p2 = __shfl(pre[2], b >> 2, 64), p3 = __shfl(pre[3], b >> 2, 64);
      const unsigned p = (b & 3) == 0 ? p0 : (b & 3) == 1 ? p1 : (b & 3) == 2 ? p2 : p3;
      if (e < e1) ((int*)B.order)[p + (key & ((1u << DX_OKEY_RANK_BITS) - 1u))] = e;
    }
  }
  // 2. the deferred physics steps.  Beside a mid-tier launch: first the step kernel's
  // deferrals the mid tier has not taken (it may not have run yet: a profiler or a shared
  // hardware queue can serialise the streams), from their hand-off records; then, once
  // every one of them has finished (the mid tier's too), those beyond the mid tier's pool
  const unsigned n1 = B.mid ? B.defer[0] : 0u;
  for (unsigned i = blockIdx.x; i < n1; i += gridDim.x) {
    unsigned e = 0;
    int got = 0;
    if (LANE == 0) {
      got = defer_claim(B.defer, i, &e);
      if (got == 1) atomicAdd(B.health + 8, 1u);  // a step-kernel deferral the mid tier did not take
    }
    if (__shfl(got, 0, 64) != 1) continue;
    e = __shfl(e, 0, 64);
    const int env = defer_env(e), s0 = defer_step(e);
    CtxT<SpecRT> c(m, L, smem, nullptr, nullptr);
    c.I = (int*)(smem + c.L.ints);
    c.sep = B.sepcache ? B.sepcache + (size_t)env * DX_SEP_SLOTS : nullptr;
    c.np_wide = B.np_wide;
    float time = env_begin(c, B, env, B.hand + (size_t)env * B.hand_stride, true);
    for (int s = s0; s < nsub; s++) env_substep(c, B, time, env, s == nsub - 1);
    env_finish(c, B, env, time);
    if (B.fuse) fused_post(c, B, env, false);
    if (LANE == 0) __hip_atomic_fetch_add(B.qdone + 1, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
  int ok = 1;
  if (B.mid) {
    if (LANE == 0) {
      for (unsigned w = 0; __hip_atomic_load(B.qdone + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < n1; w++) {
        __builtin_amdgcn_s_sleep(4);
        if (w > (1u << 25)) { __hip_atomic_store(B.qerr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); ok = 0; break; }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    ok = __shfl(ok, 0, 64);
  }
  // (a timed-out wait skips the second list -- its entries may not be complete; qerr[0]
  // reports the launch -- but still counts this workgroup below, so the last one resets
  // the launch-to-launch state and later launches start from clean lists)
  unsigned* list = B.mid ? B.defer2 : B.defer;
  const unsigned n = list && ok ? list[0] : 0u;
  for (unsigned i = blockIdx.x; i < n; i += gridDim.x) {
    const unsigned e = list[2 + i];
    const int env = defer_env(e), s0 = defer_step(e);
    CtxT<SpecRT> c(m, L, smem, nullptr, nullptr);
    c.I = (int*)(smem + c.L.ints);
    c.sep = B.sepcache ? B.sepcache + (size_t)env * DX_SEP_SLOTS : nullptr;
    c.np_wide = B.np_wide;
    float time = env_begin(c, B, env, nullptr, true);
    if (e & DX_DEFER_FWD) {
      forward(c, B.xfrc);
      if (B.sen_stash) sensor_stash(c, B, env);
      health_check(c, B, env, time, false);
      env_finish(c, B, env, time);
    } else {
      for (int s = s0; s < nsub; s++) env_substep(c, B, time, env, s == nsub - 1);
      env_finish(c, B, env, time);
      if (B.fuse) fused_post(c, B, env, false);
    }
  }
  // 3. the last workgroup to finish resets the launch-to-launch state
  unsigned last = 0;
  if (LANE == 0) {
    __threadfence();
    last = atomicAdd((unsigned*)B.qerr + 1, 1u) == gridDim.x - 1;
  }
  if (__shfl(last, 0, 64)) {
    __threadfence();
    // the deferral lists: entries, counts, the finished count
    for (unsigned i = LANE; B.defer && i < B.defer[0]; i += DX_WAVE) B.defer[2 + i] = 0u;
    for (unsigned i = LANE; B.defer2 && i < B.defer2[0]; i += DX_WAVE) B.defer2[2 + i] = 0u;
    SYNC();
    if (B.defer && LANE < 2) B.defer[LANE] = 0u;
    if (B.defer2 && LANE < 2) B.defer2[LANE] = 0u;
    if (B.qdone && LANE == 0) B.qdone[1] = 0u;
    if (B.onext)                                           // this launch's cost histogram
#pragma unroll
      for (int k = 0; k < 4; k++) B.ohist[256 * B.opar + 4 * LANE + k] = 0u;
    if (LANE < DX_QUEUES) B.qhead[LANE * DX_QHEAD_STRIDE] = 0u;  // the queue heads
    if (LANE == 0) B.qerr[1] = 0u;
  }
}

hipError_t dx_launch_step_hi(int grid, size_t lds, hipStream_t stream, const DevModel* m, const DevBatch& B,
                             const Lds& L, int nsub) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)dx_step_hi_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  hipLaunchKernelGGL(dx_step_hi_kernel, dim3(grid), dim3(64), lds, stream, m, B, L, nsub);
  return hipGetLastError();
}
#elif defined(DX_TIER_MID)
// ------------------------------------------------------------------------ //
// mid tier (build.py compiles this file once more with -DDX_TIER_MID
// -DDX_NCON_MAX=DX_NCON_MID): launched on a side stream beside a queued step-kernel launch
// of nslot workgroups (one slot short of the chip's, so one CU keeps room for this
// workgroup's LDS), it takes the physics steps the step kernel defers while that launch
// runs -- instead of after it, on an otherwise idle chip -- and runs each deferred env
// from its hand-off record to the end of its control step with the DX_NCON_MID pool, with
// the step kernel's outputs and task logic.  A physics step beyond this pool goes on to
// the overflow tier's list (B.defer2).  Entries are taken in order by compare-and-swap
// (defer_claim), as the overflow tier takes any the mid tier has not when it runs after
// the launch; the overflow tier's last workgroup zeroes them for the next launch.  The
// launch's end is its workgroups' exit count (B.qdone[0], never reset) reaching `target`;
// after it every entry below the count is taken.  No stream event joins the two streams:
// each finished entry counts in B.qdone[1] (release), and the overflow tier waits until
// every entry of the launch has finished (acquire) -- it never waits for the mid tier to
// start, so a serialised order cannot deadlock.  The waits are bounded (B.qerr).
// ------------------------------------------------------------------------ //
static_assert(DX_NCON_MAX == DX_NCON_MID, "the mid tier is compiled with the DX_NCON_MID pool");
extern "C" __global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2)))
dx_step_mid_kernel(const DevModel* __restrict__ mp, DevBatch B, Lds L, int nsub, unsigned target) {
  extern __shared__ float smem[];
  const DevModel& m = *(const DevModel*)(const DXG DevModel*)mp;
  for (unsigned i = 0;;) {
    unsigned e = 0;
    int got = 0;
    if (LANE == 0) {
      unsigned last = ~0u;
      for (unsigned n = 0;; n++) {
        const unsigned qd = __hip_atomic_load(B.qdone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const bool done = (int)(qd - target) >= 0;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned cnt = __hip_atomic_load(B.defer, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (i < cnt) {
          const int r = defer_claim(B.defer, i, &e, B.epoch);
          if (r == 1) { got = 1; break; }
          if (r == 2) { i++; continue; }  // the overflow tier took it
        } else if (done) {
          break;  // the launch is over and every deferral below cnt was taken
        }
        __builtin_amdgcn_s_sleep(4);
        // Giving up is always safe -- the overflow tier takes every entry left -- so the
        // wait sets no error: it ends a mid tier that runs before its launch's step kernel
        // (a profiler serialising the dispatches) or one whose launch aborted.  The clock
        // restarts whenever the launch finishes a task, so a long launch (CG, PGS: 5-18 ms)
        // keeps its mid tier; ~14 ms without one finished task ends the wait.  Counted in
        // health word 7 (speed only: the entries then run behind the launch).
        if (qd != last) { last = qd; n = 0; }
        if (++n > (1u << 17) || ((n & 1023u) == 0 && __hip_atomic_load(B.qerr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
          atomicAdd(B.health + 7, 1u);
          break;
        }
      }
    }
    i = __shfl(i, 0, 64);
    if (!__shfl(got, 0, 64)) break;
    e = __shfl(e, 0, 64);
    i++;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int env = defer_env(e), s0 = defer_step(e);
    CtxT<SpecRT> c(m, L, smem, nullptr, nullptr);
    c.I = (int*)(smem + c.L.ints);
    c.sep = B.sepcache ? B.sepcache + (size_t)env * DX_SEP_SLOTS : nullptr;
    c.np_wide = B.np_wide;
    c.defer = true;
    c.defer_at = B.mid_defer_at;
    const float* rec = B.hand + (size_t)env * B.hand_stride;
    float time = env_begin(c, B, env, rec, true);
    int s = s0;
    for (; s < nsub; s++) {
      env_substep(c, B, time, env, s == nsub - 1);
      if (c.I[I_DEFER]) break;
    }
    if (s < nsub) {
      env_defer(c, B, env, s, false, time, B.defer2);
    } else {
      env_finish(c, B, env, time);
      if (B.fuse) fused_post(c, B, env, false);
    }
    // finished: its stores (and a deferral to the overflow tier's list) before the count
    // the overflow tier waits for
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (LANE == 0) __hip_atomic_fetch_add(B.qdone + 1, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}

hipError_t dx_launch_step_mid(int grid, size_t lds, hipStream_t stream, const DevModel* m, const DevBatch& B,
                              const Lds& L, int nsub, unsigned target) {
  hipLaunchKernelGGL(dx_step_mid_kernel, dim3(grid), dim3(64), lds, stream, m, B, L, nsub, target);
  return hipGetLastError();
}
#elif defined(DX_SPEC_ONLY)
#define DX_SPEC_DEFINE(SP)                                                                            \
  bool dx_match_##SP(const DevModel& d, const Lds& L) { return spec_matches<SP>(d, L); }             \
  int dx_occ_##SP(size_t lds) {                                                                       \
    int n = 0;                                                                                        \
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, dx_step_kernel_queue_spec<SP>, 64, lds) != hipSuccess) n = 0; \
    return n;                                                                                         \
  }                                                                                                   \
  hipError_t dx_launch_##SP(int grid, size_t lds, hipStream_t stream, const DevModel* m, const DevBatch& B, \
                            const Lds& L, int nsub, int mode) {                                       \
    if (mode == 2)                                                                                    \
      hipLaunchKernelGGL(dx_prep_kernel_spec<SP>, dim3(grid), dim3(64), lds, stream, m, B, L);         \
    else if (mode == 3)                                                                               \
      hipLaunchKernelGGL(dx_step_kernel_queue_spec<SP>, dim3(grid), dim3(64), lds, stream, m, B, L, nsub);  \
    else                                                                                              \
      hipLaunchKernelGGL(dx_step_kernel_spec<SP>, dim3(grid), dim3(64), lds, stream, m, B, L, nsub, mode); \
    return hipGetLastError();                                                                         \
  }
#define DX_SPEC_DEFINE1(SP) DX_SPEC_DEFINE(SP)
DX_SPEC_DEFINE1(DX_SPEC_ONLY)
#else
DX_SPECS(DX_SPEC_FNS)

// The model struct is read through a device pointer (dx_api.hip device_model) in
// the constant address space rather than passed by value in the kernarg segment.
extern "C" __global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(DX_STEP_WAVES)))
dx_step_kernel(const DevModel* __restrict__ mp, DevBatch B, Lds L, int nsub, int mode) {
  const DevModel& m = *(const DevModel*)(const DXG DevModel*)mp;
  if (mode == 3) step_queue<SpecRT>(m, B, L, nsub);
  else step_body<SpecRT>(m, B, L, nsub, mode);
}
extern "C" __global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2)))
dx_prep_kernel(const DevModel* __restrict__ mp, DevBatch B, Lds L) {
  const DevModel& m = *(const DevModel*)(const DXG DevModel*)mp;
  step_body<SpecRT>(m, B, L, 1, 2, true);
}

// Resident step-kernel workgroups per CU at `lds` bytes of LDS each (0: unknown), for
// the persistent grid of the substep queue.
int dx_step_occupancy(int spec, size_t lds) {
  int k = 0;
#define DX_OCC(SP) if (spec == k) return dx_occ_##SP(lds); k++;
  DX_SPECS(DX_OCC)
#undef DX_OCC
  (void)k;
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, dx_step_kernel, 64, lds) != hipSuccess) n = 0;
  return n;
}

// Whether specialization `spec` carries the fused reach sampling pass (fused_reach_prep).
bool dx_spec_reach(int spec) {
  int k = 0;
#define DX_REACH(SP) if (spec == k) return SP::reach_task; k++;
  DX_SPECS(DX_REACH)
#undef DX_REACH
  (void)k;
  return false;
}

// Index of the specialization whose layout and dimensions equal the model's, or -1.
int dx_spec_find(const DevModel& d, const Lds& L) {
  int k = 0;
#define DX_TRY(SP) if (dx_match_##SP(d, L)) return k; k++;
  DX_SPECS(DX_TRY)
#undef DX_TRY
  (void)k;
  return -1;
}

// Longest-processing-time-first dispatch order: a counting sort of the envs by their
// last step's cost (descending, 256 buckets of 16 K shader cycles), one workgroup.
// The order within a bucket depends on atomic timing, which only changes which CU
// runs an environment, never its results.
// The same kernel zeroes the substep-queue heads for the next launch (qhead != nullptr):
// no separate memset node per step.
__global__ void __launch_bounds__(1024) dx_order_kernel(int nenv, const unsigned* cost, int* order, unsigned* qhead) {
  __shared__ int hist[256];
  __shared__ int base[256];
  const int t = threadIdx.x;
  if (t < 256) hist[t] = 0;
  if (qhead && t < DX_QUEUES) qhead[t * DX_QHEAD_STRIDE] = 0u;
  __syncthreads();
  for (int e = t; e < nenv; e += 1024) atomicAdd(&hist[255 - (int)min(cost[e] >> 4, 255u)], 1);
  __syncthreads();
  if (t < 64) {  // exclusive prefix of the 256 buckets: four per lane, then a wave scan
    const int h0 = hist[4 * t], h1 = hist[4 * t + 1], h2 = hist[4 * t + 2], h3 = hist[4 * t + 3];
    const int tot = h0 + h1 + h2 + h3;
    const int ex = wave_incl_scan(tot) - tot;
    base[4 * t] = ex;
    base[4 * t + 1] = ex + h0;
    base[4 * t + 2] = ex + h0 + h1;
    base[4 * t + 3] = ex + h0 + h1 + h2;
  }
  __syncthreads();
  for (int e = t; e < nenv; e += 1024) order[atomicAdd(&base[255 - (int)min(cost[e] >> 4, 255u)], 1)] = e;
}

hipError_t dx_launch_order(int nenv, hipStream_t stream, const unsigned* cost, int* order, unsigned* qhead) {
  hipLaunchKernelGGL(dx_order_kernel, dim3(1), dim3(1024), 0, stream, nenv, cost, order, qhead);
  return hipGetLastError();
}

hipError_t dx_launch_step(int spec, int grid, size_t lds, hipStream_t stream, const DevModel* m, const DevBatch& B,
                          const Lds& L, int nsub, int mode) {
  int k = 0;
#define DX_LAUNCH(SP)                                                         \
  if (spec == k) return dx_launch_##SP(grid, lds, stream, m, B, L, nsub, mode); \
  k++;
  DX_SPECS(DX_LAUNCH)
#undef DX_LAUNCH
  (void)k;
  if (mode == 2)
    hipLaunchKernelGGL(dx_prep_kernel, dim3(grid), dim3(64), lds, stream, m, B, L);
  else
    hipLaunchKernelGGL(dx_step_kernel, dim3(grid), dim3(64), lds, stream, m, B, L, nsub, mode);
  return hipGetLastError();
}

// reset envs [env0, env0+n) to qpos0
extern "C" __global__ void dx_reset_kernel(DevModel m, DevBatch B, int env0, int n) {
  int env = env0 + blockIdx.x;
  if (blockIdx.x >= n || env >= B.nenv) return;
  for (int i = LANE; i < m.nq; i += blockDim.x) B.qpos[(size_t)env * m.nq + i] = m.qpos0[i];
  for (int i = LANE; i < m.nv; i += blockDim.x) {
    B.qvel[(size_t)env * m.nv + i] = 0;
    B.qacc_ws[(size_t)env * m.nv + i] = 0;
    B.qacc[(size_t)env * m.nv + i] = 0;
  }
  for (int i = LANE; i < m.nu; i += blockDim.x) B.ctrl[(size_t)env * m.nu + i] = 0;
  if (LANE == 0) {
    B.time[env] = 0;
    if (B.nstep) B.nstep[env] = 0;
  }
}
#endif  // DX_TIER_HI / DX_TIER_MID / DX_SPEC_ONLY
