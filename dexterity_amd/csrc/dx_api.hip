// dx_api.hip -- host implementation of include/dx.h.
//
// dx_model_load parses the compiled-model blob (fp64 arrays from the build-time
// compiler), derives the tables the kernels index (tree levels, dof chain
// bitmasks, friction/limit row maps, dense fixed-tendon Jacobians), converts to
// fp32 and uploads one read-only copy per device.  dx_batch owns the per-env
// state arrays ([nenv][width], fp32) and a HIP stream.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <map>
#include <string>
#include <vector>

#include "../../include/dx.h"
#include "dx_internal.h"

extern "C" __global__ void dx_step_kernel(const DevModel* mp, DevBatch B, Lds L, int nsub, int mode);
extern "C" __global__ void dx_reset_kernel(DevModel m, DevBatch B, int env0, int n);

static thread_local std::string g_err;
static int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
#define HIPCHK(x)                                                                          \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) return fail(DX_EHIP, std::string(#x ": ") + hipGetErrorString(e_)); \
  } while (0)

extern "C" const char* dx_last_error(void) { return g_err.c_str(); }
extern "C" int dx_abi_version(void) { return DX_ABI_VERSION; }

// ------------------------------------------------------------------------ //
// blob parsing
// ------------------------------------------------------------------------ //
struct BlobArr {
  int dtype;
  long n;
  const void* p;
};

static bool parse_blob(const unsigned char* b, size_t nbytes, std::map<std::string, BlobArr>& out) {
  if (nbytes < 16 || memcmp(b, "DXMBLOB1", 8) != 0) return false;
  long n;
  memcpy(&n, b + 8, 8);
  if (n < 0 || 16 + n * 72 > (long)nbytes) return false;
  for (long i = 0; i < n; i++) {
    const unsigned char* e = b + 16 + i * 72;
    char name[49];
    memcpy(name, e, 48);
    name[48] = 0;
    int code;
    long cnt, off;
    memcpy(&code, e + 48, 4);
    memcpy(&cnt, e + 56, 8);
    memcpy(&off, e + 64, 8);
    size_t esz = code == 0 ? 4 : 8;
    if (off < 0 || cnt < 0 || (size_t)off + cnt * esz > nbytes) return false;
    out[name] = BlobArr{code, cnt, b + off};
  }
  return true;
}

struct dx_model {
  std::vector<unsigned char> blob;
  std::map<std::string, BlobArr> arr;
  // host copies (fp32 / int) of every device array, keyed by name
  std::map<std::string, std::vector<float>> hf;
  std::map<std::string, std::vector<int>> hi;
  std::vector<uint64_t> body_chain;
  DevModel dm;  // host-side scalars; pointers filled per device
  std::map<int, std::vector<void*>> dev_allocs;
  std::map<int, DevModel> dev_models;
  std::map<int, const DevModel*> dev_model_ptrs;  // device copy of dev_models[device]
  Lds lds;     // the step kernel's per-env LDS layout (contact pool DX_NCON_MAX)
  Lds lds_hi;  // the overflow tier's (DX_NCON_HI)
  Lds lds_mid; // the mid tier's (DX_NCON_MID; nefc_max 0: not available for this model)
  int ncon_max, nefc_max;
};

static int geti(const dx_model* m, const char* name, int def = -1) {
  auto it = m->arr.find(name);
  if (it == m->arr.end() || it->second.dtype != 0 || it->second.n < 1) return def;
  return ((const int*)it->second.p)[0];
}
static double getd(const dx_model* m, const char* name, double def = 0) {
  auto it = m->arr.find(name);
  if (it == m->arr.end() || it->second.dtype != 1 || it->second.n < 1) return def;
  return ((const double*)it->second.p)[0];
}
static bool load_f(dx_model* m, const char* name) {
  auto it = m->arr.find(name);
  if (it == m->arr.end() || it->second.dtype != 1) return false;
  const double* p = (const double*)it->second.p;
  m->hf[name].assign(p, p + it->second.n);
  return true;
}
static bool load_i(dx_model* m, const char* name) {
  auto it = m->arr.find(name);
  if (it == m->arr.end() || it->second.dtype != 0) return false;
  const int* p = (const int*)it->second.p;
  m->hi[name].assign(p, p + it->second.n);
  return true;
}
static void quat2mat_h(float* R, const float* q) {
  float w = q[0], x = q[1], y = q[2], z = q[3];
  R[0] = 1 - 2 * (y * y + z * z); R[1] = 2 * (x * y - w * z); R[2] = 2 * (x * z + w * y);
  R[3] = 2 * (x * y + w * z); R[4] = 1 - 2 * (x * x + z * z); R[5] = 2 * (y * z - w * x);
  R[6] = 2 * (x * z - w * y); R[7] = 2 * (y * z + w * x); R[8] = 1 - 2 * (x * x + y * y);
}


// ------------------------------------------------------------------------ //
// direction-binned hulls (support-point acceleration, exact)
// ------------------------------------------------------------------------ //
// A hull with more than DX_HULL_K (8) vertices gets a cube map of n x n cells per face
// over the local direction sphere (cell rule: dx_step.hip hull_cell).  Each cell lists
// the vertices that can be a support point for some direction in the cell, sorted by
// vertex index.  A vertex is dropped only if a single other vertex beats it by more
// than 1e-5 R at all four corner directions of the (slightly enlarged) cell, hence at
// every direction of the cell: every maximiser -- ties included -- of every direction
// in the cell is kept, and the lowest-index maximiser over the cell's list is the
// vertex the full scan returns (the oracle's rule).
// Layout: one DX_HULL_K-slot block per cell (x, y, z, vertex index; index -1 pads) -- one
// 128-B line, read by a lane group in one memory round trip of one or two 16-B loads per
// lane.  A cell with more than K candidates (the faces of a hull with many coplanar
// vertices: all of them tie along the face normal) keeps candidates 0..K-2 in its block
// and a header in slot K-1 = (overflow offset in float4s from the hull's first cell,
// candidate count, 0, index -2); candidates K-1.. follow in the hull's overflow run,
// padded to a multiple of K.  n is the smallest of 1, 2, 3, 4, 6, 8, 10, 12 with at most
// 2 % of the cells overflowing.  (Round 6: 8-slot cells on finer maps instead of 16-slot
// cells -- half the loads and candidate tests per support, one line per cell.)
static void cell_corners(int face, int n, int iu, int iv, double eps, double c[4][3]) {
  int ax = face >> 1;
  double sgn = (face & 1) ? -1.0 : 1.0;
  double u0 = -1 + 2.0 * iu / n - eps, u1 = -1 + 2.0 * (iu + 1) / n + eps;
  double v0 = -1 + 2.0 * iv / n - eps, v1 = -1 + 2.0 * (iv + 1) / n + eps;
  double us[4] = {u0, u1, u1, u0}, vs[4] = {v0, v0, v1, v1};
  for (int k = 0; k < 4; k++) {
    c[k][ax] = sgn;
    c[k][(ax + 1) % 3] = us[k];
    c[k][(ax + 2) % 3] = vs[k];
  }
}

static void hull_cell_candidates(const std::vector<double>& V, int nv, double R, const double c[4][3],
                                 std::vector<int>& out) {
  std::vector<double> D(4 * nv), S(nv);
  for (int i = 0; i < nv; i++) {
    for (int k = 0; k < 4; k++)
      D[4 * i + k] = V[3 * i] * c[k][0] + V[3 * i + 1] * c[k][1] + V[3 * i + 2] * c[k][2];
    S[i] = D[4 * i] + D[4 * i + 1] + D[4 * i + 2] + D[4 * i + 3];
  }
  std::vector<int> order(nv);
  for (int i = 0; i < nv; i++) order[i] = i;
  std::sort(order.begin(), order.end(), [&](int a, int b) { return S[a] > S[b]; });
  double cn[4];
  for (int k = 0; k < 4; k++) cn[k] = std::sqrt(c[k][0] * c[k][0] + c[k][1] * c[k][1] + c[k][2] * c[k][2]);
  const double tol = 1e-5 * R;
  out.clear();
  for (int v = 0; v < nv; v++) {
    bool dominated = false;
    for (int w : order) {
      if (S[w] <= S[v]) break;  // a dominator beats v at every corner, so also in the sum
      bool all = true;
      for (int k = 0; k < 4 && all; k++) all = D[4 * w + k] - D[4 * v + k] > tol * cn[k];
      if (all) { dominated = true; break; }
    }
    if (!dominated) out.push_back(v);
  }
}

static void build_hull_bins(dx_model* m) {
  auto& mv = m->hf["mesh_vert"];
  auto& adr = m->hi["mesh_vertadr"];
  auto& num = m->hi["mesh_vertnum"];
  int nmesh = (int)num.size();
  std::vector<int> bn(std::max(nmesh, 1), 0), bcap(std::max(nmesh, 1), 0), badr(std::max(nmesh, 1), 0);
  std::vector<float> b4;
  static const int kN[] = {1, 2, 3, 4, 6, 8, 10, 12};
  constexpr int K = DX_HULL_K;
  const char* env_minn = getenv("DX_HULL_BIN_MINN");  // (experiments: finer cube maps)
  const int minn = env_minn ? atoi(env_minn) : 1;
  for (int i = 0; i < nmesh; i++) {
    int nv = num[i];
    if (nv <= K) continue;
    std::vector<double> V(3 * nv);
    double R = 0;
    for (int j = 0; j < nv; j++) {
      for (int k = 0; k < 3; k++) V[3 * j + k] = mv[3 * (adr[i] + j) + k];
      R = std::max(R, std::sqrt(V[3 * j] * V[3 * j] + V[3 * j + 1] * V[3 * j + 1] + V[3 * j + 2] * V[3 * j + 2]));
    }
    std::vector<std::vector<int>> cells;
    int n = 0;
    for (int nn : kN) {
      if (nn < minn && nn != kN[7]) continue;
      cells.assign(6 * nn * nn, {});
      int over = 0;
      for (int f = 0; f < 6; f++)
        for (int iu = 0; iu < nn; iu++)
          for (int iv = 0; iv < nn; iv++) {
            double c[4][3];
            cell_corners(f, nn, iu, iv, 1e-3, c);
            auto& L = cells[(f * nn + iu) * nn + iv];
            hull_cell_candidates(V, nv, R, c, L);
            over += L.size() > K;
          }
      n = nn;
      if (over <= 0.02 * (double)cells.size()) break;
    }
    const size_t base = b4.size() / 4;  // this hull's first cell, in float4s
    const size_t ncell = cells.size();
    b4.resize(4 * (base + K * ncell), 0.f);
    auto put = [&](size_t slot, int idx) {
      float* e = b4.data() + 4 * slot;
      for (int k = 0; k < 3; k++) e[k] = idx >= 0 ? mv[3 * (adr[i] + idx) + k] : 0.f;
      memcpy(e + 3, &idx, 4);
    };
    for (size_t cidx = 0; cidx < ncell; cidx++) {
      const auto& L = cells[cidx];
      const size_t blk = base + K * cidx;
      if (L.size() <= (size_t)K) {
        for (int s = 0; s < K; s++) put(blk + s, s < (int)L.size() ? L[s] : -1);
        continue;
      }
      for (int s = 0; s < K - 1; s++) put(blk + s, L[s]);
      const size_t ov = b4.size() / 4;  // overflow run: candidates K-1.., padded to K
      const int nov = (int)L.size() - (K - 1);
      b4.resize(4 * (ov + (size_t)(nov + K - 1) / K * K), 0.f);
      for (int s = 0; s < (nov + K - 1) / K * K; s++) put(ov + s, s < nov ? L[K - 1 + s] : -1);
      float* h = b4.data() + 4 * (blk + K - 1);
      const int off = (int)(ov - base), cnt = (int)L.size(), tag = -2;
      memcpy(h, &off, 4);
      memcpy(h + 1, &cnt, 4);
      h[2] = 0.f;
      memcpy(h + 3, &tag, 4);
    }
    bn[i] = n;
    bcap[i] = K;
    badr[i] = (int)base;
  }
  if (b4.empty()) b4.assign(4, 0.f);
  m->hf["mesh_bin4"] = b4;
  m->hi["mesh_binn"] = bn;
  m->hi["mesh_bincap"] = bcap;
  m->hi["mesh_binadr"] = badr;
}

static const char* kFloatArrays[] = {
    "body_pos", "body_quat", "body_ipos", "body_iquat", "body_mass", "body_inertia", "body_bsphere",
    "body_invweight0", "jnt_pos", "jnt_axis", "jnt_range", "jnt_margin", "jnt_solref", "jnt_solimp",
    "qpos0", "dof_armature", "dof_damping", "dof_frictionloss", "dof_solref", "dof_solimp",
    "dof_invweight0", "geom_size", "geom_pos", "geom_quat", "geom_center", "geom_bsphere", "geom_aabb", "mesh_vert",
    "site_pos", "site_quat", "tendon_range", "tendon_margin", "tendon_solref", "tendon_solimp",
    "tendon_invweight0", "wrap_coef", "actuator_gear", "actuator_gainprm", "actuator_biasprm",
    "actuator_ctrlrange", "actuator_forcerange", "gpair_friction", "gpair_solref", "gpair_solimp",
    "gpair_margin", "gravity", "bpair_sphere"};
static const char* kIntArrays[] = {
    "body_parent", "body_rootid", "body_jntnum", "body_jntadr", "body_dofnum", "body_dofadr",
    "jnt_type", "jnt_bodyid", "jnt_qposadr", "jnt_dofadr", "jnt_limited", "dof_bodyid",
    "dof_parentid", "dof_jntid", "geom_type", "geom_bodyid", "geom_dataid", "mesh_vertadr",
    "mesh_vertnum", "site_bodyid", "tendon_adr", "tendon_num", "tendon_limited", "wrap_dof",
    "actuator_trntype", "actuator_trnid", "actuator_biastype", "actuator_ctrllimited",
    "actuator_forcelimited", "bpair_body", "bpair_adr", "bpair_num", "bpair_plane", "gpair_geom", "gpair_condim"};

extern "C" dx_model* dx_model_load(const void* blob, size_t nbytes) {
  if (!blob) { fail(DX_EINVAL, "null blob"); return nullptr; }
  dx_model* m = new dx_model();
  m->blob.assign((const unsigned char*)blob, (const unsigned char*)blob + nbytes);
  if (!parse_blob(m->blob.data(), nbytes, m->arr)) {
    fail(DX_EMODEL, "malformed model blob");
    delete m;
    return nullptr;
  }
  for (const char* n : kFloatArrays)
    if (!load_f(m, n)) { fail(DX_EMODEL, std::string("blob missing float array ") + n); delete m; return nullptr; }
  for (const char* n : kIntArrays)
    if (!load_i(m, n)) { fail(DX_EMODEL, std::string("blob missing int array ") + n); delete m; return nullptr; }
  DevModel& d = m->dm;
  memset(&d, 0, sizeof(d));
  d.nq = geti(m, "nq"); d.nv = geti(m, "nv"); d.nbody = geti(m, "nbody"); d.njnt = geti(m, "njnt");
  d.ngeom = geti(m, "ngeom"); d.nsite = geti(m, "nsite"); d.nu = geti(m, "nu");
  d.ntendon = geti(m, "ntendon"); d.nwrap = geti(m, "nwrap"); d.nbpair = geti(m, "nbpair");
  d.ngpair = geti(m, "ngpair"); d.iterations = geti(m, "iterations");
  d.disable_contact = geti(m, "disable_contact");
  d.solver = geti(m, "solver", 2);  // absent in every reference scene: MuJoCo's default, Newton
  if (d.solver < 0 || d.solver > 2) {
    fail(DX_EMODEL, "unknown solver");
    delete m;
    return nullptr;
  }
  d.timestep = (float)getd(m, "timestep"); d.tolerance = (float)getd(m, "tolerance");
  d.impratio = (float)getd(m, "impratio"); d.meaninertia = (float)getd(m, "meaninertia");
  for (int k = 0; k < 3; k++) d.gravity[k] = m->hf["gravity"][k];
  if (d.nv < 1 || d.nv > DX_MAX_NV || d.nbody < 1) {
    fail(DX_ELIMIT, "nv must be in [1, 64]");
    delete m;
    return nullptr;
  }
  if (d.nu > 64 || d.njnt > 64) {  // one lane per actuator / joint (velocity stage, Euler)
    fail(DX_ELIMIT, "nu and njnt must be <= 64");
    delete m;
    return nullptr;
  }
  int nb = d.nbody, nv = d.nv;
  auto& parent = m->hi["body_parent"];
  auto& rootid = m->hi["body_rootid"];
  // roots, levels
  std::vector<int> rootidx(nb, 0), roots;
  for (int b = 1; b < nb; b++) {
    if (parent[b] == 0) { rootidx[b] = (int)roots.size(); roots.push_back(b); }
  }
  for (int b = 1; b < nb; b++) rootidx[b] = rootidx[rootid[b]];
  std::vector<int> depth(nb, 0);
  int maxd = 0;
  for (int b = 1; b < nb; b++) { depth[b] = depth[parent[b]] + 1; maxd = std::max(maxd, depth[b]); }
  std::vector<int> lvl_adr(maxd + 1, 0), lvl_body;
  for (int lv = 1; lv <= maxd; lv++) {
    lvl_adr[lv - 1] = (int)lvl_body.size();
    for (int b = 1; b < nb; b++)
      if (depth[b] == lv) lvl_body.push_back(b);
  }
  lvl_adr[maxd] = (int)lvl_body.size();
  d.nlevel = maxd;
  d.nroot = (int)roots.size();
  m->hi["body_rootidx"] = rootidx;
  m->hi["root_body"] = roots.empty() ? std::vector<int>{0} : roots;
  m->hi["lvl_adr"] = lvl_adr;
  m->hi["lvl_body"] = lvl_body.empty() ? std::vector<int>{0} : lvl_body;
  // dof chain masks
  m->body_chain.assign(nb, 0);
  auto& dofadr = m->hi["body_dofadr"];
  auto& dofnum = m->hi["body_dofnum"];
  for (int b = 1; b < nb; b++) {
    uint64_t c = m->body_chain[parent[b]];
    for (int k = 0; k < dofnum[b]; k++) c |= 1ull << (dofadr[b] + k);
    m->body_chain[b] = c;
  }
  // check contact jacobian support limit over all candidate body pairs
  auto& bpair = m->hi["bpair_body"];
  for (int k = 0; k < d.nbpair; k++) {
    uint64_t s = m->body_chain[bpair[2 * k]] ^ m->body_chain[bpair[2 * k + 1]];
    if (__builtin_popcountll(s) > DX_DOFMAX) {
      fail(DX_ELIMIT, "contact jacobian support exceeds DX_DOFMAX");
      delete m;
      return nullptr;
    }
  }
  // rotation matrices
  auto mats = [&](const char* qname, const char* out, int n) {
    std::vector<float> R(9 * std::max(n, 1), 0.f);
    auto& q = m->hf[qname];
    for (int i = 0; i < n; i++) quat2mat_h(R.data() + 9 * i, q.data() + 4 * i);
    m->hf[out] = R;
  };
  mats("body_iquat", "body_imat", nb);
  mats("geom_quat", "geom_mat", d.ngeom);
  mats("site_quat", "site_mat", d.nsite);
  {
    // (x, y, z, the vertex's index in its mesh as int bits): a whole-hull scan reads the
    // index from the slot as a cell scan does, so every support load is one 16-B load
    auto& mv = m->hf["mesh_vert"];
    std::vector<float> v4(4 * std::max<size_t>(mv.size() / 3, 1), 0.f);
    for (size_t i = 0; i < mv.size() / 3; i++)
      for (int k = 0; k < 3; k++) v4[4 * i + k] = mv[3 * i + k];
    auto& vadr = m->hi["mesh_vertadr"];
    auto& vnum = m->hi["mesh_vertnum"];
    for (size_t g = 0; g < vnum.size(); g++)
      for (int j = 0; j < vnum[g]; j++) memcpy(&v4[4 * ((size_t)vadr[g] + j) + 3], &j, 4);
    m->hf["mesh_vert4"] = v4;
  }
  build_hull_bins(m);
  // per-geom shape records and per-pair records for the narrowphase setup: one or two
  // memory round trips instead of a chain of dependent table lookups
  {
    auto& gt = m->hi["geom_type"]; auto& gb = m->hi["geom_bodyid"]; auto& gdid = m->hi["geom_dataid"];
    auto& gs = m->hf["geom_size"]; auto& gp = m->hf["geom_pos"]; auto& gm = m->hf["geom_mat"];
    auto& gc = m->hf["geom_center"];
    auto& vadr = m->hi["mesh_vertadr"]; auto& vnum = m->hi["mesh_vertnum"];
    auto& bn = m->hi["mesh_binn"]; auto& bc = m->hi["mesh_bincap"]; auto& ba = m->hi["mesh_binadr"];
    int ng = (int)gt.size();
    std::vector<float> rec(32 * std::max(ng, 1), 0.f);
    for (int g = 0; g < ng; g++) {
      float* r = rec.data() + 32 * g;
      int iv[8] = {gt[g], gb[g], 0, 0, 0, 0, 0, 0};
      if (gt[g] == DXG_MESH) {
        int mid = gdid[g];
        iv[2] = vnum[mid]; iv[3] = bn[mid]; iv[4] = bc[mid]; iv[5] = vadr[mid]; iv[6] = ba[mid];
      }
      memcpy(r, iv, sizeof(iv));
      for (int k = 0; k < 3; k++) { r[8 + k] = gs[3 * g + k]; r[12 + k] = gp[3 * g + k]; r[25 + k] = gc[3 * g + k]; }
      for (int k = 0; k < 9; k++) r[16 + k] = gm[9 * g + k];
    }
    m->hf["geom_rec"] = rec;
    auto& pg = m->hi["gpair_geom"]; auto& pm = m->hf["gpair_margin"];
    int np = (int)pm.size();
    std::vector<float> prec(4 * std::max(np, 1), 0.f);
    for (int k = 0; k < np; k++) {
      int g1 = pg[2 * k], g2 = pg[2 * k + 1];
      int prim = gt[g1] == DXG_PLANE || (gt[g1] == DXG_CAPSULE && gt[g2] == DXG_CAPSULE);
      int iv[2] = {g1, g2};
      memcpy(&prec[4 * k], iv, 8);
      prec[4 * k + 2] = pm[k];
      memcpy(&prec[4 * k + 3], &prim, 4);
    }
    m->hf["gpair_rec"] = prec;
  }

  // geom bounding spheres with centres in the body frame (mid-phase cull)
  {
    std::vector<float> gb(4 * std::max(d.ngeom, 1), 0.f);
    auto& gs = m->hf["geom_bsphere"];
    auto& gp = m->hf["geom_pos"];
    auto& gm = m->hf["geom_mat"];
    for (int g = 0; g < d.ngeom; g++) {
      const float* R = gm.data() + 9 * g;
      const float* cc = gs.data() + 4 * g;
      for (int k = 0; k < 3; k++)
        gb[4 * g + k] = gp[3 * g + k] + R[3 * k] * cc[0] + R[3 * k + 1] * cc[1] + R[3 * k + 2] * cc[2];
      gb[4 * g + 3] = cc[3];
    }
    m->hf["geom_bsphere_b"] = gb;
    // oriented bounding box in the body frame: centre(3), R(9) body<-box, half extents(3)
    std::vector<float> ob(15 * std::max(d.ngeom, 1), 0.f);
    auto& ga = m->hf["geom_aabb"];
    for (int g = 0; g < d.ngeom; g++) {
      const float* R = gm.data() + 9 * g;
      const float* a = ga.data() + 6 * g;
      for (int k = 0; k < 3; k++)
        ob[15 * g + k] = gp[3 * g + k] + R[3 * k] * a[0] + R[3 * k + 1] * a[1] + R[3 * k + 2] * a[2];
      for (int k = 0; k < 9; k++) ob[15 * g + 3 + k] = R[k];
      for (int k = 0; k < 3; k++) ob[15 * g + 12 + k] = a[3 + k];
    }
    m->hf["geom_obb_b"] = ob;
  }
  // collision culling records: per geom {type, body}{bsphere (body frame)}{obb centre,
  // R (body <- box), half extents; planes: point, normal} and per body pair {b1, b2,
  // first geom pair, count}{sphere 1}{sphere 2}{margin, plane geom, plane body, box
  // margin}{plane point | box 1 centre, half x}{plane normal | box 1 half y z, box 2
  // centre x y}{box 2 centre z, half extents} (body frames) -- one memory round trip
  // per culling item
  {
    auto& gt = m->hi["geom_type"]; auto& gb = m->hi["geom_bodyid"];
    auto& gbs = m->hf["geom_bsphere_b"]; auto& gob = m->hf["geom_obb_b"];
    auto& gp = m->hf["geom_pos"]; auto& gm = m->hf["geom_mat"];
    int ng = (int)gt.size();
    std::vector<float> cr(24 * std::max(ng, 1), 0.f);
    for (int g = 0; g < ng; g++) {
      float* r = cr.data() + 24 * g;
      int iv[2] = {gt[g], gb[g]};
      memcpy(r, iv, 8);
      for (int k = 0; k < 4; k++) r[4 + k] = gbs[4 * g + k];
      if (gt[g] == DXG_PLANE) {
        for (int k = 0; k < 3; k++) { r[8 + k] = gp[3 * g + k]; r[20 + k] = gm[9 * g + 3 * k + 2]; }
      } else {
        for (int k = 0; k < 3; k++) r[8 + k] = gob[15 * g + k];
        for (int k = 0; k < 9; k++) r[11 + k] = gob[15 * g + 3 + k];
        for (int k = 0; k < 3; k++) r[20 + k] = gob[15 * g + 12 + k];
      }
    }
    m->hf["geom_crec"] = cr;
    auto& bb = m->hi["bpair_body"]; auto& ba = m->hi["bpair_adr"]; auto& bnum = m->hi["bpair_num"];
    auto& bpl = m->hi["bpair_plane"]; auto& bs = m->hf["bpair_sphere"]; auto& pm = m->hf["gpair_margin"];
    int nbp = (int)bnum.size();
    auto& gpg = m->hi["gpair_geom"];
    std::vector<float> br(28 * std::max(nbp, 1), 0.f);
    for (int k = 0; k < nbp; k++) {
      float* r = br.data() + 28 * k;
      int iv[4] = {bb[2 * k], bb[2 * k + 1], ba[k], bnum[k]};
      memcpy(r, iv, 16);
      for (int e = 0; e < 8; e++) r[4 + e] = bs[8 * k + e];
      r[12] = pm[ba[k]];
      int pg = bpl[k], pb = pg >= 0 ? gb[pg] : 0;
      memcpy(r + 13, &pg, 4);
      memcpy(r + 14, &pb, 4);
      if (pg >= 0) {
        for (int e = 0; e < 3; e++) { r[16 + e] = gp[3 * pg + e]; r[20 + e] = gm[9 * pg + 3 * e + 2]; }
      } else {
        // Box cull: per side, the body-frame box around the OBBs (geom_obb_b) of that
        // side's geoms in this pair, grown by a little, and the largest geom-pair
        // margin.  Geom pairs whose OBBs overlap have overlapping boxes, so a pair the
        // boxes separate has no geom pair the mid-phase would keep.
        double lo[2][3] = {{1e30, 1e30, 1e30}, {1e30, 1e30, 1e30}};
        double hi[2][3] = {{-1e30, -1e30, -1e30}, {-1e30, -1e30, -1e30}};
        double mmax = 0;
        for (int q = ba[k]; q < ba[k] + bnum[k]; q++) {
          mmax = std::max(mmax, (double)pm[q]);
          for (int t = 0; t < 2; t++) {
            int g = gpg[2 * q + t];
            int side = gb[g] == bb[2 * k] ? 0 : 1;
            const float* o = gob.data() + 15 * g;
            for (int cnr = 0; cnr < 8; cnr++) {
              double sgn[3] = {(cnr & 1) ? 1.0 : -1.0, (cnr & 2) ? 1.0 : -1.0, (cnr & 4) ? 1.0 : -1.0};
              for (int i = 0; i < 3; i++) {
                double v = o[i];
                for (int jj = 0; jj < 3; jj++) v += (double)o[3 + 3 * i + jj] * sgn[jj] * o[12 + jj];
                lo[side][i] = std::min(lo[side][i], v);
                hi[side][i] = std::max(hi[side][i], v);
              }
            }
          }
        }
        float c[2][3], e[2][3];
        for (int side = 0; side < 2; side++)
          for (int i = 0; i < 3; i++) {
            c[side][i] = (float)(0.5 * (lo[side][i] + hi[side][i]));
            e[side][i] = (float)(0.5 * (hi[side][i] - lo[side][i]) * (1.0 + 1e-4) + 1e-5);
          }
        r[15] = (float)mmax;
        const float rec[12] = {c[0][0], c[0][1], c[0][2], e[0][0], e[0][1], e[0][2],
                               c[1][0], c[1][1], c[1][2], e[1][0], e[1][1], e[1][2]};
        for (int i = 0; i < 12; i++) r[16 + i] = rec[i];
      }
    }
    m->hf["bpair_rec"] = br;
  }
  // tree records: per body (lane = body in the level loops) and per dof, so a stage
  // loads its model data in one memory round trip instead of a chain per tree level
  if (nb > 64) {
    fail(DX_ELIMIT, "nbody must be <= 64 (one lane per body)");
    delete m;
    return nullptr;
  }
  {
    auto& bja = m->hi["body_jntadr"]; auto& bjn = m->hi["body_jntnum"];
    auto& jt = m->hi["jnt_type"]; auto& jqa = m->hi["jnt_qposadr"]; auto& jda = m->hi["jnt_dofadr"];
    auto& bpos = m->hf["body_pos"]; auto& bquat = m->hf["body_quat"]; auto& bipos = m->hf["body_ipos"];
    auto& jpos = m->hf["jnt_pos"]; auto& jax = m->hf["jnt_axis"]; auto& q0 = m->hf["qpos0"];
    auto& bmass = m->hf["body_mass"]; auto& binert = m->hf["body_inertia"];
    std::vector<float> br(32 * nb, 0.f);
    for (int b = 0; b < nb; b++) {
      float* r = br.data() + 32 * b;
      int ja = bja[b], jn = bjn[b];
      int iv0[4] = {parent[b], depth[b], ja, jn};
      memcpy(r, iv0, 16);
      int jtp = jn > 0 ? jt[ja] : -1, qa = jn > 0 ? jqa[ja] : 0, jd = jn > 0 ? jda[ja] : 0;
      for (int k = 0; k < 3; k++) { r[4 + k] = bpos[3 * b + k]; r[12 + k] = bipos[3 * b + k]; }
      memcpy(r + 7, &jtp, 4);
      for (int k = 0; k < 4; k++) r[8 + k] = bquat[4 * b + k];
      memcpy(r + 15, &rootidx[b], 4);
      if (jn > 0)
        for (int k = 0; k < 3; k++) { r[16 + k] = jpos[3 * ja + k]; r[20 + k] = jax[3 * ja + k]; }
      memcpy(r + 19, &qa, 4);
      r[23] = jn > 0 ? q0[qa] : 0.f;
      int iv6[2] = {dofadr[b], dofnum[b]};
      memcpy(r + 24, iv6, 8);
      r[26] = bmass[b];
      memcpy(r + 27, &jd, 4);
      for (int k = 0; k < 3; k++) r[28 + k] = binert[3 * b + k];
    }
    m->hf["body_rec"] = br;
    auto& dbody = m->hi["dof_bodyid"]; auto& djnt = m->hi["dof_jntid"];
    auto& arm = m->hf["dof_armature"]; auto& dmp = m->hf["dof_damping"];
    std::vector<float> dr(8 * nv, 0.f);
    for (int d2 = 0; d2 < nv; d2++) {
      float* r = dr.data() + 8 * d2;
      int b = dbody[d2], j = djnt[d2];
      int tk = jt[j] | ((d2 - jda[j]) << 8);
      int iv[4] = {b, j, rootidx[b], tk};
      memcpy(r, iv, 16);
      r[4] = arm[d2];
      r[5] = dmp[d2];
      uint64_t anc = m->body_chain[b] & ((d2 >= 63) ? ~0ull : ((2ull << d2) - 1ull));
      uint32_t lo = (uint32_t)anc, hi = (uint32_t)(anc >> 32);
      memcpy(r + 6, &lo, 4);
      memcpy(r + 7, &hi, 4);
    }
    m->hf["dof_rec"] = dr;
  }
  {
    // Tree-sparse LDL^T of M (dx_device.h tree_solve): the elimination items (k, i, j)
    // -- dof k, a proper ancestor i of k, j = i or an ancestor of i -- grouped by the
    // height of k above the leaves (a level's dofs are never ancestors of one another),
    // each level padded to whole 64-item slots; bit s of ldl_sync closes a level at
    // slot s.  Deeper trees than DX_LDL_SLOTS slots keep the dense solver (nslot 0).
    auto& par = m->hi["dof_parentid"];
    std::vector<int> height(nv, 0);
    for (int k = nv - 1; k >= 0; k--)
      if (par[k] >= 0) height[par[k]] = std::max(height[par[k]], height[k] + 1);
    int hmax = 0;
    for (int k = 0; k < nv; k++) hmax = std::max(hmax, height[k]);
    std::vector<int> tab;
    unsigned sync = 0;
    int nslot = 0;
    for (int h = 0; h <= hmax; h++) {
      std::vector<int> items;
      for (int k = 0; k < nv; k++) {
        if (height[k] != h) continue;
        for (int i = par[k]; i >= 0; i = par[i])
          for (int j = i; j >= 0; j = par[j]) items.push_back(k | (i << 8) | (j << 16));
      }
      if (items.empty()) continue;
      const int ns = ((int)items.size() + DX_WAVE - 1) / DX_WAVE;
      items.resize((size_t)ns * DX_WAVE, -1);
      tab.insert(tab.end(), items.begin(), items.end());
      nslot += ns;
      if (nslot <= 32) sync |= 1u << (nslot - 1);
    }
    const char* dense = getenv("DX_DENSE_MSOLVE");  // A/B switch: the matrix-core Cholesky
    if (nslot > DX_LDL_SLOTS || nv > DX_MAX_NV || (dense && dense[0] == '1')) { nslot = 0; sync = 0; tab.clear(); }
    d.ldl_nslot = nslot;
    d.ldl_sync = sync;
    m->hi["ldl_tab"] = tab;
  }
  // friction rows / limited joints / limited tendons
  std::vector<int> fric_dof, dof_fricrow(nv, -1), limj, limt;
  auto& floss = m->hf["dof_frictionloss"];
  for (int i = 0; i < nv; i++)
    if (floss[i] > 0) { dof_fricrow[i] = (int)fric_dof.size(); fric_dof.push_back(i); }
  auto& jtype = m->hi["jnt_type"];
  auto& jlim = m->hi["jnt_limited"];
  for (int j = 0; j < d.njnt; j++)
    if (jlim[j] && jtype[j] == DXJ_HINGE) limj.push_back(j);
  auto& tlim = m->hi["tendon_limited"];
  for (int t = 0; t < d.ntendon; t++)
    if (tlim[t]) limt.push_back(t);
  d.nfric = (int)fric_dof.size();
  d.nlimj = (int)limj.size();
  d.nlimt = (int)limt.size();
  m->hi["fric_dof"] = fric_dof.empty() ? std::vector<int>{0} : fric_dof;
  m->hi["dof_fricrow"] = dof_fricrow;
  m->hi["limj_jnt"] = limj.empty() ? std::vector<int>{0} : limj;
  m->hi["limt_ten"] = limt.empty() ? std::vector<int>{0} : limt;
  // wraps: qpos address; dense tendon jacobian
  auto& wdof = m->hi["wrap_dof"];
  auto& dofj = m->hi["dof_jntid"];
  auto& jqa = m->hi["jnt_qposadr"];
  std::vector<int> wqadr(std::max(d.nwrap, 1), 0);
  for (int w = 0; w < d.nwrap; w++) wqadr[w] = jqa[dofj[wdof[w]]];
  m->hi["wrap_qadr"] = wqadr;
  std::vector<float> tJ(std::max(d.ntendon, 1) * nv, 0.f);
  auto& tadr = m->hi["tendon_adr"];
  auto& tnum = m->hi["tendon_num"];
  auto& wcoef = m->hf["wrap_coef"];
  for (int t = 0; t < d.ntendon; t++)
    for (int w = tadr[t]; w < tadr[t] + tnum[t]; w++) tJ[t * nv + wdof[w]] += wcoef[w];
  m->hf["tendon_J"] = tJ;
  auto& damp = m->hf["dof_damping"];
  d.any_damping = 0;
  for (int i = 0; i < nv; i++)
    if (damp[i] > 0) d.any_damping = 1;
  // LDS layout (4-byte words).  Persistent arrays first, then a union whose
  // contents change with the stage (dx_step.hip forward()):
  //   A  kinematic block      xpos xmat xipos rcom cdof   kinematics .. make_constraint
  //   B1 com temporaries      cinert cvel cdof_dot scr xanchor xaxis xquat
  //                                                       kinematics .. velocity stage
  //   B2 smooth-solve transpose (packed nv x nv)          smooth solve
  //   B3 candidate lists + hull staging                   collision
  //   B4 constraint rows + contact jacobians              make_constraint .. qfrc_constraint
  //   H  Newton Hessian / Euler transpose over A          solve, euler
  // The union keeps one environment in < 20 KB for the Shadow scene, so eight
  // 64-lane workgroups (two waves per SIMD) fit in a CU's 160 KB.
  auto layout = [&](int cap, Lds& L) {
  int off = 0;
  auto take = [&](int n) { int o = off; off += (n + 3) & ~3; return o; };
  auto r4 = [](int n) { return (n + 3) & ~3; };
  const int ntri = nv * (nv + 1) / 2;
  L.ints = take(16);
  L.qpos = take(d.nq); L.qvel = take(nv); L.ctrl = take(std::max(d.nu, 1)); L.qacc = take(nv);
  L.qacc_smooth = take(nv); L.qfrc_smooth = take(nv); L.qfrc_con = take(nv);
  L.v1 = take(nv); L.v2 = take(nv); L.v3 = take(nv); L.v4 = take(nv); L.v5 = take(nv);
  L.M = take(ntri);
  L.ten_len = take(std::max(d.ntendon, 1));  // read by the tendon-limit rows: persistent
  L.con = take((cap + DX_NCON_SPARE) * DX_CON_STRIDE);
  // limit rows: a joint / tendon whose range is wider than twice its margin can have only
  // one side within the margin at a time (q - lo < margin and hi - q < margin need
  // hi - lo < 2 margin), so it holds one row, else two
  int nlimrow = 0;
  {
    auto& jr = m->hf["jnt_range"]; auto& jm = m->hf["jnt_margin"];
    for (int j : limj) nlimrow += (jr[2 * j + 1] - jr[2 * j]) > 2.0f * jm[j] + 1e-4f ? 1 : 2;
    auto& tr = m->hf["tendon_range"]; auto& tm = m->hf["tendon_margin"];
    for (int t : limt) nlimrow += (tr[2 * t + 1] - tr[2 * t]) > 2.0f * tm[t] + 1e-4f ? 1 : 2;
  }
  L.nefc_max = d.nfric + nlimrow + 4 * cap;
  L.efc_fl = take(std::max(d.nfric, 1)); L.efc_Rf = take(std::max(d.nfric, 1));
  L.tri = 0;  // (was the wave Cholesky's index table; n > 32 now factors on the matrix cores)
  const int U0 = off;
  L.xpos = take(3 * nb); L.xmat = take(9 * nb); L.xipos = take(3 * nb);
  L.rcom = take(3 * std::max(d.nroot, 1)); L.cdof = take(6 * nv);
  const int B0 = off;
  L.cinert = take(10 * nb); L.cvel = take(6 * nb); L.cdof_dot = take(6 * nv); L.scr = take(12 * nb);
  L.xanchor = take(3 * std::max(d.njnt, 1)); L.xaxis = take(3 * std::max(d.njnt, 1));
  L.xquat = take(4 * nb);
  // actuator lengths: tendon_lengths -> the velocity stage's actuator forces
  L.act_len = take(std::max(d.nu, 1));
  L.act_force = L.act_len;  // (no longer stored)
  int end = off;
  L.tsm = B0;
  end = std::max(end, B0 + r4(ntri));
  L.cand_max = DX_CAND_MAX;
  L.cand = B0;
  // + MPR portal points of up to DX_NGRP_MAX narrowphase groups (36 words each), then the
  // candidates' pair records (float4 per candidate slot: cand_max - 2 * (cand_max / 3))
  end = std::max(end, L.cand + L.cand_max + DX_NGRP_MAX * 36 + 4 * (L.cand_max - 2 * (L.cand_max / 3)));
  off = std::max(B0, U0 + r4(ntri));
  L.efc_meta = take(L.nefc_max); L.efc_D = take(L.nefc_max); L.efc_aref = take(L.nefc_max);
  L.efc_jar = take(L.nefc_max);
  L.cj_idx = take((cap * DX_DOFMAX + 3) / 4);  // uint8 dof ids
  L.cj_val = take(cap * 3 * DX_DOFMAX);
  // contact-frame scratch: J x in jac_vec, the frame forces in jac_t_force (and the
  // sensor stash right after the last one); never live at the same time
  L.cq = take(3 * cap);
  L.cw = L.cq;
  // The solver's J dir (efc_jv) and CG's M^-1 grad (PGS's M^-1 J_r'): written only from
  // the solve on, when the kinematic block is dead, so they go past the Newton Hessian
  // when it has room
  int spare = U0 + r4(ntri);
  if (spare + r4(L.nefc_max) <= B0) { L.efc_jv = spare; spare += r4(L.nefc_max); }
  else L.efc_jv = take(L.nefc_max);
  if (d.solver == 2) L.cgv = 0;  // Newton: no CG / PGS scratch
  else if (spare + r4(nv) <= B0) L.cgv = spare;
  else L.cgv = take(nv);
  end = std::max(end, off);
  L.H = U0;
  L.total = (end + 3) & ~3;  // the kernels zero it with 16-byte stores
  };
  // the step kernel's layout (pool DX_NCON_MAX) and the overflow tier's (DX_NCON_HI)
  layout(DX_NCON_MAX, m->lds);
  layout(DX_NCON_HI, m->lds_hi);
  layout(DX_NCON_MID, m->lds_mid);
  if (m->lds_mid.nefc_max > 5 * 64) m->lds_mid.nefc_max = 0;  // (its line search keeps 5 register slots)
  if (getenv("DX_PRINT_LDS"))
    fprintf(stderr, "dx: LDS per env %d B (step kernel), %d B (mid tier), %d B (overflow tier)\n", m->lds.total * 4,
            m->lds_mid.total * 4, m->lds_hi.total * 4);
  // the contact tiers exist only for a model that can have contacts (dx_batch_create
  // allocates the deferral lists and launches the tiers for those only): a contact-free
  // model is held to the step kernel's layout alone
  const bool tiers = !d.disable_contact && d.ngpair > 0;
  m->ncon_max = tiers ? DX_NCON_HI : DX_NCON_MAX;
  m->nefc_max = tiers ? m->lds_hi.nefc_max : m->lds.nefc_max;
  // line-search register slots (dx_step.hip DX_LS_SLOTS: 5 in the step kernel, 20 in the
  // overflow tier)
  if (m->lds.nefc_max > 5 * 64 || (tiers && m->lds_hi.nefc_max > 20 * 64)) {
    fail(DX_ELIMIT, "constraint row capacity exceeds the line search's register slots");
    delete m;
    return nullptr;
  }
  if (m->lds.total * 4 > 160 * 1024 || (tiers && m->lds_hi.total * 4 > 160 * 1024)) {
    fail(DX_ELIMIT, "per-env LDS footprint exceeds 160 KiB");
    delete m;
    return nullptr;
  }
  return m;
}

extern "C" void dx_model_free(dx_model* m) {
  if (!m) return;
  for (auto& kv : m->dev_allocs) {
    int cur;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(kv.first);
    for (void* p : kv.second) (void)hipFree(p);
    (void)hipSetDevice(cur);
  }
  delete m;
}

extern "C" int dx_model_sizes(const dx_model* m, int32_t out[12]) {
  if (!m || !out) return fail(DX_EINVAL, "null argument");
  const DevModel& d = m->dm;
  int v[12] = {d.nq, d.nv, d.nbody, d.njnt, d.ngeom, d.nsite, d.nu, d.ntendon, d.nbpair, d.ngpair,
               m->ncon_max, m->nefc_max};
  memcpy(out, v, sizeof(v));
  return 0;
}

// Host twin of the device's binned support scan (test hook): the vertex index the
// kernel's support_grp returns for hull `mesh` along local direction dir, plus the
// mesh's cube-map resolution and cell capacity (0, 0 when the hull is not binned).
extern "C" int dx_hull_support(const dx_model* m, int32_t mesh, const float dir[3], int32_t info[3]) {
  if (!m || !dir || !info) return fail(DX_EINVAL, "null argument");
  auto& num = m->hi.at("mesh_vertnum");
  if (mesh < 0 || mesh >= (int)num.size()) return fail(DX_EINVAL, "mesh out of range");
  int n = m->hi.at("mesh_binn")[mesh], cap = m->hi.at("mesh_bincap")[mesh];
  const float* b4 = m->hf.at("mesh_bin4").data() + 4 * (size_t)m->hi.at("mesh_binadr")[mesh];
  const float* mv = m->hf.at("mesh_vert").data() + 3 * (size_t)m->hi.at("mesh_vertadr")[mesh];
  int best = -1;
  float bd = -3.0e38f;
  int cell = -1;
  if (n > 0) {
    float ax0 = std::fabs(dir[0]), ax1 = std::fabs(dir[1]), ax2 = std::fabs(dir[2]);
    int ax = (ax0 >= ax1 && ax0 >= ax2) ? 0 : (ax1 >= ax2 ? 1 : 2);
    float a = dir[ax], u = dir[(ax + 1) % 3], v = dir[(ax + 2) % 3];
    if (std::fabs(a) > 1e-30f) {
      float inv = 1.0f / std::fabs(a);
      int iu = std::min(std::max((int)((u * inv + 1.0f) * 0.5f * (float)n), 0), n - 1);
      int iv = std::min(std::max((int)((v * inv + 1.0f) * 0.5f * (float)n), 0), n - 1);
      cell = ((2 * ax + (a < 0 ? 1 : 0)) * n + iu) * n + iv;
    }
  }
  if (cell >= 0) {
    // the cell's block, then its overflow run when slot K - 1 is a header
    const int K = cap;
    const float* blk = b4 + 4 * (size_t)cell * K;
    int hdr;
    memcpy(&hdr, blk + 4 * (K - 1) + 3, 4);
    int off = 0, cnt = K;
    if (hdr == -2) { memcpy(&off, blk + 4 * (K - 1), 4); memcpy(&cnt, blk + 4 * (K - 1) + 1, 4); }
    for (int s = 0; s < cnt; s++) {
      const float* e = hdr == -2 && s >= K - 1 ? b4 + 4 * ((size_t)off + s - (K - 1)) : blk + 4 * s;
      int idx;
      memcpy(&idx, e + 3, 4);
      if (idx < 0) continue;
      float d = e[0] * dir[0] + e[1] * dir[1] + e[2] * dir[2];
      if (d > bd) { bd = d; best = idx; }
    }
  } else {
    for (int i = 0; i < num[mesh]; i++) {
      float d = mv[3 * i] * dir[0] + mv[3 * i + 1] * dir[1] + mv[3 * i + 2] * dir[2];
      if (d > bd) { bd = d; best = i; }
    }
  }
  info[0] = best;
  info[1] = n;
  info[2] = cap;
  return 0;
}

// Layout export for build.py's kernel specialization: the Lds struct (words, in
// declaration order) followed by the 17 dimensions of dx_device.h DX_DIMS.
extern "C" int dx_model_layout(const dx_model* m, int32_t* out, int32_t n) {
  if (!m || !out) return fail(DX_EINVAL, "null argument");
  const int nl = (int)(sizeof(Lds) / sizeof(int));
  const DevModel& d = m->dm;
  int dims[17] = {d.nq, d.nv, d.nbody, d.njnt, d.nu, d.ntendon, d.nsite, d.nlevel, d.nroot,
                  d.nfric, d.nlimj, d.nlimt, d.nbpair, d.any_damping, d.disable_contact, d.iterations, d.solver};
  if (n < nl + 17) return fail(DX_EINVAL, "output too small");
  memcpy(out, &m->lds, sizeof(Lds));
  memcpy(out + nl, dims, sizeof(dims));
  return nl + 17;
}

extern "C" int dx_model_lds_bytes(const dx_model* m) {
  if (!m) return fail(DX_EINVAL, "null model");
  return m->lds.total * 4;
}

extern "C" int dx_field_width(const dx_model* m, int field) {
  if (!m) return fail(DX_EINVAL, "null model");
  const DevModel& d = m->dm;
  switch (field) {
    case DX_QPOS: return d.nq;
    case DX_QVEL: case DX_QACC_WARMSTART: case DX_QACC: return d.nv;
    case DX_CTRL: return d.nu;
    case DX_TIME: case DX_NCON: case DX_GROUND_CONTACT: case DX_NITER: case DX_NCAND: case DX_STEP_COST:
    case DX_DIVERGED: return 1;
    case DX_SITE_XPOS: return 3 * d.nsite;
    case DX_SITE_VEL: return 6 * d.nsite;
    case DX_XPOS: return 3 * d.nbody;
    case DX_XQUAT: return 4 * d.nbody;
    case DX_SENSOR_TORQUE: return 3 * d.nbody;
  }
  return fail(DX_EINVAL, "unknown field");
}

// Upload the model to `device` once; returns the DevModel with device pointers.
static int device_model(dx_model* m, int device, DevModel* out) {
  auto it = m->dev_models.find(device);
  if (it != m->dev_models.end()) { *out = it->second; return 0; }
  DevModel d = m->dm;
  std::vector<void*>& allocs = m->dev_allocs[device];
  auto upf = [&](const char* name, const void** dst) -> int {
    auto& v = m->hf[name];
    size_t n = std::max<size_t>(v.size(), 1);
    void* p = nullptr;
    HIPCHK(hipMalloc(&p, n * 4));
    allocs.push_back(p);
    if (!v.empty()) HIPCHK(hipMemcpy(p, v.data(), v.size() * 4, hipMemcpyHostToDevice));
    *dst = p;
    return 0;
  };
  auto upi = [&](const char* name, const void** dst) -> int {
    auto& v = m->hi[name];
    size_t n = std::max<size_t>(v.size(), 1);
    void* p = nullptr;
    HIPCHK(hipMalloc(&p, n * 4));
    allocs.push_back(p);
    if (!v.empty()) HIPCHK(hipMemcpy(p, v.data(), v.size() * 4, hipMemcpyHostToDevice));
    *dst = p;
    return 0;
  };
#define UF(field) { const void* p_; if (int rc = upf(#field, &p_)) return rc; d.field = (decltype(d.field))p_; }
#define UI(field) { const void* p_; if (int rc = upi(#field, &p_)) return rc; d.field = (decltype(d.field))p_; }
  UI(body_parent); UI(body_rootidx); UI(body_jntnum); UI(body_jntadr); UI(body_dofnum); UI(body_dofadr);
  UI(lvl_adr); UI(lvl_body); UI(root_body);
  UF(body_pos); UF(body_quat); UF(body_ipos); UF(body_imat); UF(body_mass); UF(body_inertia);
  UF(body_bsphere); UF(body_invweight0);
  UI(jnt_type); UI(jnt_bodyid); UI(jnt_qposadr); UI(jnt_dofadr);
  UF(jnt_pos); UF(jnt_axis); UF(jnt_range); UF(jnt_margin); UF(jnt_solref); UF(jnt_solimp); UF(qpos0);
  UI(limj_jnt); UI(dof_bodyid); UI(dof_parentid); UI(dof_jntid); UI(fric_dof); UI(dof_fricrow);
  UF(dof_armature); UF(dof_damping); UF(dof_frictionloss); UF(dof_solref); UF(dof_solimp); UF(dof_invweight0);
  UI(geom_type); UI(geom_bodyid); UI(geom_dataid);
  UF(geom_size); UF(geom_pos); UF(geom_mat); UF(geom_center); UF(geom_bsphere); UF(geom_bsphere_b); UF(geom_obb_b);
  UI(mesh_vertadr); UI(mesh_vertnum); UF(mesh_vert4);
  UI(mesh_binn); UI(mesh_bincap); UI(mesh_binadr); UF(mesh_bin4);
  UF(geom_rec); UF(gpair_rec); UF(geom_crec); UF(bpair_rec); UF(body_rec); UF(dof_rec); UI(ldl_tab);
  UI(site_bodyid); UF(site_pos); UF(site_mat);
  UI(tendon_adr); UI(tendon_num); UI(wrap_dof); UI(wrap_qadr); UI(limt_ten);
  UF(tendon_range); UF(tendon_margin); UF(tendon_solref); UF(tendon_solimp); UF(tendon_invweight0);
  UF(wrap_coef); UF(tendon_J);
  UI(actuator_trntype); UI(actuator_trnid); UI(actuator_biastype); UI(actuator_ctrllimited);
  UI(actuator_forcelimited);
  UF(actuator_gear); UF(actuator_gainprm); UF(actuator_biasprm); UF(actuator_ctrlrange); UF(actuator_forcerange);
  UI(bpair_body); UI(bpair_adr); UI(bpair_num); UI(bpair_plane); UF(bpair_sphere); UI(gpair_geom); UI(gpair_condim);
  UF(gpair_friction); UF(gpair_solref); UF(gpair_solimp); UF(gpair_margin);
#undef UF
#undef UI
  void* p = nullptr;
  HIPCHK(hipMalloc(&p, m->body_chain.size() * 8));
  allocs.push_back(p);
  HIPCHK(hipMemcpy(p, m->body_chain.data(), m->body_chain.size() * 8, hipMemcpyHostToDevice));
  d.body_chain = (decltype(d.body_chain))p;
  // the struct itself, for the kernels that read the model through a pointer
  HIPCHK(hipMalloc(&p, sizeof(DevModel)));
  allocs.push_back(p);
  HIPCHK(hipMemcpy(p, &d, sizeof(DevModel), hipMemcpyHostToDevice));
  m->dev_model_ptrs[device] = (const DevModel*)p;
  m->dev_models[device] = d;
  *out = d;
  return 0;
}

// ------------------------------------------------------------------------ //
// batch
// ------------------------------------------------------------------------ //
struct dx_batch {
  dx_model* model;
  int device, nenv;
  hipStream_t stream;
  DevModel dm;
  const DevModel* dm_dev;  // the same struct in device memory (kernels read it through this)
  DevBatch db;
  int spec;  // specialized step kernel (dx_specs.inc) or -1 for the generic one
  bool queue;  // mode-0 steps through the substep queue
  bool qhead_zero = false;  // the last kernel on the stream zeroed the queue heads
  int* watch_list = nullptr;  // device copy of DevBatch::watch_pairs
  int slots;   // persistent workgroups of a queued launch
  int hi_grid; // workgroups of the overflow tier's launch
  float* xfrc;
  std::vector<void*> allocs;
  bool debug;
  float* sensor = nullptr;  // DX_SENSOR_TORQUE [nenv][nbody][3] (allocated by dx_sensor_enable)
  float* sen_stash = nullptr;
  unsigned* ncon_hist = nullptr;  // dx_ncon_histogram
  // the mid tier beside queued launches (dx_step.hip dx_step_mid_kernel): its stream, the
  // queued workgroups' exit count it waits for (DevBatch::qdone[0])
  bool mid = false;
  hipStream_t side = nullptr;
  unsigned qdone_target = 0;
};

#define DX_HI_GRID 32  // workgroups of the overflow tier (each loops over the deferred steps)

static int balloc(dx_batch* b, void** p, size_t bytes) {
  HIPCHK(hipMalloc(p, std::max<size_t>(bytes, 4)));
  HIPCHK(hipMemsetAsync(*p, 0, std::max<size_t>(bytes, 4), b->stream));
  b->allocs.push_back(*p);
  return 0;
}

extern "C" dx_batch* dx_batch_create(const dx_model* mc, int32_t nenv, int32_t device) {
  dx_model* m = const_cast<dx_model*>(mc);
  if (!m || nenv < 1) { fail(DX_EINVAL, "bad model or nenv"); return nullptr; }
  if (nenv > (1 << DX_DEFER_ENV_BITS)) { fail(DX_ELIMIT, "nenv above 2^20 per batch (deferral entries)"); return nullptr; }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) {
    fail(DX_EHIP, "invalid HIP device (is a GPU visible?)");
    return nullptr;
  }
  if (hipSetDevice(device) != hipSuccess) { fail(DX_EHIP, "hipSetDevice failed"); return nullptr; }
  dx_batch* b = new dx_batch();
  b->model = m;
  b->device = device;
  b->nenv = nenv;
  b->debug = false;
  b->xfrc = nullptr;
  if (hipStreamCreateWithFlags(&b->stream, hipStreamNonBlocking) != hipSuccess) {
    fail(DX_EHIP, "hipStreamCreate failed");
    delete b;
    return nullptr;
  }
  if (device_model(m, device, &b->dm) != 0) { delete b; return nullptr; }
  b->dm_dev = m->dev_model_ptrs[device];
  b->spec = getenv("DX_GENERIC_KERNEL") ? -1 : dx_spec_find(b->dm, m->lds);
  const DevModel& d = b->dm;
  DevBatch& B = b->db;
  memset(&B, 0, sizeof(B));
  B.nenv = nenv;
  size_t E = nenv;
  int rc = 0;
  rc |= balloc(b, (void**)&B.qpos, E * d.nq * 4);
  rc |= balloc(b, (void**)&B.qvel, E * d.nv * 4);
  rc |= balloc(b, (void**)&B.ctrl, E * std::max(d.nu, 1) * 4);
  rc |= balloc(b, (void**)&B.qacc_ws, E * d.nv * 4);
  rc |= balloc(b, (void**)&B.qacc, E * d.nv * 4);
  rc |= balloc(b, (void**)&B.time, E * 4);
  rc |= balloc(b, (void**)&B.site_xpos, E * 3 * std::max(d.nsite, 1) * 4);
  rc |= balloc(b, (void**)&B.site_vel, E * 6 * std::max(d.nsite, 1) * 4);
  rc |= balloc(b, (void**)&B.xpos, E * 3 * d.nbody * 4);
  rc |= balloc(b, (void**)&B.xquat, E * 4 * d.nbody * 4);
  rc |= balloc(b, (void**)&B.ncon, E * 4);
  rc |= balloc(b, (void**)&B.watch, E * 4);
  rc |= balloc(b, (void**)&B.niter, E * 4);
  rc |= balloc(b, (void**)&B.ncand, E * 4);
  if (!getenv("DX_NO_SEPCACHE"))  // (A/B and traffic attribution: MPR without the separating-direction cache)
    rc |= balloc(b, (void**)&B.sepcache, E * DX_SEP_SLOTS * 16);
  rc |= balloc(b, (void**)&B.health, DX_HEALTH_WORDS * 4);
  rc |= balloc(b, (void**)&B.bad, E * 4);
  rc |= balloc(b, (void**)&B.nstep, E * 4);
  // the overflow tier's deferral list (models that can have contacts)
  if (!d.disable_contact && d.ngpair > 0) rc |= balloc(b, (void**)&B.defer, (E + 2) * 4);
  if (!getenv("DX_NO_LPT_ORDER")) {
    void* po = nullptr;
    rc |= balloc(b, (void**)&B.cost, E * 4);
    rc |= balloc(b, &po, E * 4);
    B.order = (const int*)po;
    rc |= balloc(b, (void**)&B.ohist, 2 * 256 * 4);
    rc |= balloc(b, (void**)&B.okey, E * 4);
  }
  rc |= balloc(b, (void**)&b->xfrc, 6 * d.nbody * 4);
  // substep queue state (DX_NO_QUEUE=1: one workgroup per env for the whole step)
  b->queue = !getenv("DX_NO_QUEUE");
  rc |= balloc(b, (void**)&B.qhead, DX_QUEUES * DX_QHEAD_STRIDE * 4);
  rc |= balloc(b, (void**)&B.progress, E * 4);
  rc |= balloc(b, (void**)&B.qerr, 8);  // [0] queue timeout, [1] the overflow kernel's finished workgroups
  B.hand_stride = (d.nq + 2 * d.nv + 4 + 31) / 32 * 32;
  rc |= balloc(b, (void**)&B.hand, E * B.hand_stride * 4);
  B.epoch = 0;
  // one queue per XCD (DX_ONE_QUEUE=1: a single queue for the whole chip)
  B.nqueue = getenv("DX_ONE_QUEUE") ? 1 : DX_QUEUES;
  B.np_wide = getenv("DX_NP_WIDE") ? atoi(getenv("DX_NP_WIDE")) : DX_WAVE / 8;
  B.defer_at = getenv("DX_DEFER_AT") ? atoi(getenv("DX_DEFER_AT")) : DX_NCON_MAX;  // (tests / probes)
  B.order_last = getenv("DX_ORDER_LAST") ? atoi(getenv("DX_ORDER_LAST")) : 1;
  b->hi_grid = getenv("DX_HI_GRID") ? std::max(1, atoi(getenv("DX_HI_GRID"))) : DX_HI_GRID;
  {
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || ncu < 1) ncu = 256;
    // resident 64-lane workgroups of the step kernel per CU (LDS and VGPR limits; 8 when
    // the runtime cannot say), plus the occupancy experiment DX_LDS_PAD (extra LDS bytes)
    const char* pad = getenv("DX_LDS_PAD");
    const size_t lds = (size_t)m->lds.total * 4 + (pad ? (size_t)atol(pad) : 0);
    int per = dx_step_occupancy(b->spec, lds);
    if (per < 1) per = (int)std::max<size_t>(1, std::min<size_t>(8, 163840 / lds));
    b->slots = ncu * per;
    // the mid tier: its workgroup fits a CU that holds one step-kernel workgroup fewer
    // (LDS in 512-B granules; its VGPRs fit the SIMD that then runs one wave)
    auto g512 = [](size_t x) { return (x + 511) / 512 * 512; };
    const size_t lmid = (size_t)m->lds_mid.total * 4;
    b->mid = b->queue && B.defer && m->lds_mid.nefc_max > 0 && !getenv("DX_NO_MID") && per >= 2 &&
             (size_t)(per - 1) * g512(lds) + g512(lmid) <= 163840;
  }
  if (b->mid) {
    rc |= balloc(b, (void**)&B.defer2, (E + 2) * 4);
    rc |= balloc(b, (void**)&B.qdone, 2 * 4);
    B.mid_defer_at = getenv("DX_MID_DEFER_AT") ? atoi(getenv("DX_MID_DEFER_AT")) : DX_NCON_MID;  // (tests)
    if (hipStreamCreateWithFlags(&b->side, hipStreamNonBlocking) != hipSuccess)
      rc |= fail(DX_EHIP, "mid-tier stream creation failed");
  }
  if (rc) { dx_batch_destroy(b); return nullptr; }
  B.xfrc = nullptr;  // enabled by dx_set_xfrc
  if (B.order && dx_launch_order(nenv, b->stream, B.cost, (int*)B.order, nullptr) != hipSuccess) {  // a permutation
    fail(DX_EHIP, "order kernel launch failed");
    dx_batch_destroy(b);
    return nullptr;
  }
  B.watch_geom = -1;
  B.watch_body = -1;
  B.out_bodies = 1;
  if (dx_reset(b, 0, nenv) != 0) { dx_batch_destroy(b); return nullptr; }
  // the mid tier's stream is ordered after nothing on the batch stream: its first launch
  // must not read the deferral list or the exit counts before their zeroing above
  if (b->mid && hipStreamSynchronize(b->stream) != hipSuccess) {
    fail(DX_EHIP, "stream sync failed");
    dx_batch_destroy(b);
    return nullptr;
  }
  return b;
}

extern "C" void dx_batch_destroy(dx_batch* b) {
  if (!b) return;
  (void)hipSetDevice(b->device);
  (void)hipStreamSynchronize(b->stream);
  if (b->side) (void)hipStreamSynchronize(b->side);
  for (void* p : b->allocs) (void)hipFree(p);
  if (b->side) (void)hipStreamDestroy(b->side);
  (void)hipStreamDestroy(b->stream);
  delete b;
}

extern "C" int dx_batch_nenv(const dx_batch* b) { return b ? b->nenv : fail(DX_EINVAL, "null batch"); }

extern "C" int dx_reset(dx_batch* b, int32_t env0, int32_t n) {
  if (!b || env0 < 0 || n < 0 || env0 + n > b->nenv) return fail(DX_EINVAL, "bad env range");
  if (n == 0) return 0;
  HIPCHK(hipSetDevice(b->device));
  hipLaunchKernelGGL(dx_reset_kernel, dim3(n), dim3(64), 0, b->stream, b->dm, b->db, env0, n);
  HIPCHK(hipGetLastError());
  return 0;
}

static void* field_base(dx_batch* b, int field) {
  DevBatch& B = b->db;
  switch (field) {
    case DX_QPOS: return B.qpos;
    case DX_QVEL: return B.qvel;
    case DX_CTRL: return B.ctrl;
    case DX_QACC_WARMSTART: return B.qacc_ws;
    case DX_QACC: return B.qacc;
    case DX_TIME: return B.time;
    case DX_SITE_XPOS: return B.site_xpos;
    case DX_SITE_VEL: return B.site_vel;
    case DX_XPOS: return B.xpos;
    case DX_XQUAT: return B.xquat;
    case DX_NCON: return B.ncon;
    case DX_GROUND_CONTACT: return B.watch;
    case DX_NITER: return B.niter;
    case DX_NCAND: return B.ncand;
    case DX_STEP_COST: return B.cost;
    case DX_SENSOR_TORQUE: return b->sensor;
    case DX_DIVERGED: return B.bad;
  }
  return nullptr;
}

// A substep-queue launch that timed out waiting for a predecessor task aborts
// (dx_step.hip step_queue); the batch state is then unusable.  Checked at every
// host synchronisation point.
static int queue_check(dx_batch* b) {
  if (!b->db.qerr) return 0;
  int err = 0;
  HIPCHK(hipMemcpy(&err, b->db.qerr, 4, hipMemcpyDeviceToHost));
  if (err) return fail(DX_EHIP, "substep queue timed out waiting for a predecessor task (launch aborted)");
  return 0;
}

extern "C" int dx_field_ptr(dx_batch* b, int field, void** devptr) {
  if (!b || !devptr) return fail(DX_EINVAL, "null argument");
  void* p = field_base(b, field);
  if (!p) return fail(DX_EINVAL, "unknown field");
  *devptr = p;
  return 0;
}

extern "C" int dx_set_field(dx_batch* b, int field, const void* src, int32_t env0, int32_t n) {
  if (!b || !src) return fail(DX_EINVAL, "null argument");
  if (env0 < 0 || n < 0 || env0 + n > b->nenv) return fail(DX_EINVAL, "bad env range");
  if (field != DX_QPOS && field != DX_QVEL && field != DX_CTRL && field != DX_QACC_WARMSTART && field != DX_TIME)
    return fail(DX_EINVAL, "field is read-only");
  int w = dx_field_width(b->model, field);
  if (w <= 0) return 0;
  char* base = (char*)field_base(b, field);
  HIPCHK(hipSetDevice(b->device));
  HIPCHK(hipMemcpyAsync(base + (size_t)env0 * w * 4, src, (size_t)n * w * 4, hipMemcpyDefault, b->stream));
  return 0;
}

extern "C" int dx_get_field(dx_batch* b, int field, void* dst, int32_t env0, int32_t n) {
  if (!b || !dst) return fail(DX_EINVAL, "null argument");
  if (env0 < 0 || n < 0 || env0 + n > b->nenv) return fail(DX_EINVAL, "bad env range");
  char* base = (char*)field_base(b, field);
  if (!base) return fail(DX_EINVAL, "unknown field");
  int w = dx_field_width(b->model, field);
  if (w <= 0) return 0;
  HIPCHK(hipSetDevice(b->device));
  HIPCHK(hipMemcpyAsync(dst, base + (size_t)env0 * w * 4, (size_t)n * w * 4, hipMemcpyDefault, b->stream));
  HIPCHK(hipStreamSynchronize(b->stream));
  return queue_check(b);
}

extern "C" int dx_set_xfrc(dx_batch* b, const float* xfrc, int32_t nbody) {
  if (!b) return fail(DX_EINVAL, "null batch");
  if (!xfrc) { b->db.xfrc = nullptr; return 0; }
  if (nbody != b->dm.nbody) return fail(DX_EINVAL, "xfrc must be [nbody][6]");
  HIPCHK(hipSetDevice(b->device));
  HIPCHK(hipMemcpyAsync(b->xfrc, xfrc, (size_t)nbody * 6 * 4, hipMemcpyDefault, b->stream));
  b->db.xfrc = b->xfrc;
  return 0;
}

static int set_watch_pairs(dx_batch* b);

extern "C" int dx_set_ground_geom(dx_batch* b, int32_t geom) {
  if (!b) return fail(DX_EINVAL, "null batch");
  if (geom >= b->dm.ngeom) return fail(DX_EINVAL, "geom out of range");
  b->db.watch_geom = geom;
  return set_watch_pairs(b);
}

// The body pairs the watch test of the observation pass has to look at: those with
// `body` on one side and the watched geom's body on the other (as filtered in
// dx_step.hip collision), listed once here instead of filtered per env and step.
static int set_watch_pairs(dx_batch* b) {
  DevBatch& B = b->db;
  std::vector<int> list;
  if (B.watch_geom >= 0 && B.watch_body >= 0) {
    const auto& bb = b->model->hi.at("bpair_body");
    const int gbody = b->model->hi.at("geom_bodyid")[B.watch_geom];
    for (int k = 0; k < b->dm.nbpair; k++) {
      const int b1 = bb[2 * k], b2 = bb[2 * k + 1];
      if ((b1 == B.watch_body || b2 == B.watch_body) && (gbody == b1 || gbody == b2)) list.push_back(k);
    }
  }
  if (!b->watch_list) {
    void* p = nullptr;
    if (balloc(b, &p, (size_t)std::max(b->dm.nbpair, 1) * 4)) return DX_EHIP;
    b->watch_list = (int*)p;
  }
  if (!list.empty())
    HIPCHK(hipMemcpyAsync(b->watch_list, list.data(), list.size() * 4, hipMemcpyHostToDevice, b->stream));
  HIPCHK(hipStreamSynchronize(b->stream));
  B.watch_pairs = b->watch_list;
  B.watch_npairs = (int)list.size();
  return 0;
}

extern "C" int dx_set_watch(dx_batch* b, int32_t geom, int32_t body) {
  if (!b) return fail(DX_EINVAL, "null batch");
  if (geom >= b->dm.ngeom || body >= b->dm.nbody) return fail(DX_EINVAL, "watch out of range");
  b->db.watch_geom = geom;
  b->db.watch_body = body;
  return set_watch_pairs(b);
}

static void timing_begin(dx_batch* b, hipEvent_t* start);
static void timing_end(dx_batch* b, hipEvent_t start);

static int launch_step(dx_batch* b, int nsub, int mode) {
  HIPCHK(hipSetDevice(b->device));
  size_t lds = (size_t)b->model->lds.total * 4;
  if (const char* pad = getenv("DX_LDS_PAD")) lds += (size_t)atol(pad);  // occupancy experiment
  // (progress tags 30 and 31 are markers: dx_step.hip DX_QUEUE_NSUB; a deferral entry
  // holds the physics step in 8 bits)
  if (b->db.defer && nsub > 255) return fail(DX_EINVAL, "at most 255 physics steps per call");
  // The substep queue pays off when the batch has more envs than the chip has wave slots
  // (heavy contact-rich envs balanced over the slots).  A contact-free batch that fits the
  // slots (Shadow reach, 1024 envs) runs one workgroup per env for the whole control step:
  // every env starts at once anyway, and its physics steps then need no hand-offs.
  const bool queued = mode == 0 && b->queue && nsub <= 29 && (b->db.defer || b->nenv > b->slots);
  // a mode-0 step builds the next launch's longest-first order, placed by the overflow
  // tier's launch (or, without one, by the order kernel)
  DevBatch& Bo = b->db;
  Bo.onext = (mode == 0 && Bo.order && Bo.defer) ? 1 : 0;
  if (Bo.onext) Bo.opar ^= 1;
  // a queued launch with the mid tier beside it leaves one workgroup slot for it
  const bool mid = queued && b->mid;
  const int grid = queued ? (int)std::min<long>((long)b->nenv * nsub, b->slots - (mid ? 1 : 0)) : b->nenv;
  if (queued) {
    // substep queue: a new progress epoch and zeroed task counters
    DevBatch& B = b->db;
    if (++B.epoch >= (1u << 26)) {  // tags wrap: start over from zeroed progress
      HIPCHK(hipMemsetAsync(B.progress, 0, (size_t)b->nenv * 4, b->stream));
      B.epoch = 1;
    }
    if (!b->qhead_zero) HIPCHK(hipMemsetAsync(B.qhead, 0, DX_QUEUES * DX_QHEAD_STRIDE * 4, b->stream));
    b->qhead_zero = false;
  }
  Bo.mid = mid ? 1 : 0;
  hipEvent_t t0;
  timing_begin(b, &t0);
  hipError_t e = dx_launch_step(b->spec, grid, lds, b->stream, b->dm_dev, b->db, b->model->lds, nsub, queued ? 3 : mode);
  timing_end(b, t0);
  HIPCHK(e);
  // the mid tier, on its own stream, with no stream event in between (dx_step.hip
  // dx_step_mid_kernel: it waits on the device for this launch's workgroups to exit, and
  // the overflow tier below waits for it).  It is submitted after the step kernel: should
  // the two streams share a hardware queue it then runs after the step kernel instead of
  // ahead of it -- the mid tier waits for the step kernel, never the other way round.
  if (mid) {
    b->qdone_target += (unsigned)grid;
    HIPCHK(dx_launch_step_mid(1, (size_t)b->model->lds_mid.total * 4, b->side, b->dm_dev, b->db, b->model->lds_mid,
                              nsub, b->qdone_target));
  }
  // the overflow tier: physics steps whose contacts did not fit the step kernel's pool
  // (nothing to do unless some env deferred one), the next launch's longest-first order,
  // and the queue heads zeroed for the next launch
  if (b->db.defer && mode != 2) {
    HIPCHK(dx_launch_step_hi(b->hi_grid, (size_t)b->model->lds_hi.total * 4, b->stream, b->dm_dev, b->db,
                             b->model->lds_hi, nsub));
    b->qhead_zero = true;
  }
  Bo.mid = 0;
  // torque sensors from the last substep's stash (mode 0 step, mode 1 forward)
  if (b->db.sen_stash && mode != 2)
    HIPCHK(dx_launch_sensor(b->nenv, ((size_t)b->model->lds.total + 6 * DX_MAX_NV) * 4, b->stream, b->dm_dev, b->db,
                            b->model->lds, b->sensor));
  // next launch: heaviest environments first (costs just measured) -- for a model without
  // an overflow tier (contacts disabled), by the order kernel, which also zeroes the queue
  // heads the next queued launch claims from
  if (mode == 0 && b->db.order && !b->db.defer && (queued || b->nenv > b->slots)) {
    HIPCHK(dx_launch_order(b->nenv, b->stream, b->db.cost, (int*)b->db.order, b->db.qhead));
    b->qhead_zero = true;
  }
  return 0;
}

// (DX_DIVERGED of a call reports that call only: the step kernel clears an env's flag in
// its first physics-step task)
extern "C" int dx_step(dx_batch* b, int32_t nsubstep) {
  if (!b || nsubstep < 1) return fail(DX_EINVAL, "bad batch or nsubstep");
  return launch_step(b, nsubstep, 0);
}

extern "C" int dx_forward(dx_batch* b) {
  if (!b) return fail(DX_EINVAL, "null batch");
  return launch_step(b, 1, 1);
}

extern "C" int dx_health(dx_batch* b, uint32_t* out, int32_t n) {
  if (!b || !out || n < 0) return fail(DX_EINVAL, "null batch or output");
  HIPCHK(hipSetDevice(b->device));
  uint32_t h[DX_HEALTH_WORDS + DX_NCON_HIST];
  memset(h, 0, sizeof(h));
  HIPCHK(hipMemcpyAsync(h, b->db.health, DX_HEALTH_WORDS * 4, hipMemcpyDeviceToHost, b->stream));
  if (b->db.ncon_hist)
    HIPCHK(hipMemcpyAsync(h + DX_HEALTH_WORDS, b->db.ncon_hist, DX_NCON_HIST * 4, hipMemcpyDeviceToHost, b->stream));
  HIPCHK(hipStreamSynchronize(b->stream));
  memcpy(out, h, std::min<size_t>(n, DX_HEALTH_WORDS + DX_NCON_HIST) * 4);
  return queue_check(b);
}

extern "C" int dx_health_clear(dx_batch* b) {
  if (!b) return fail(DX_EINVAL, "null batch");
  HIPCHK(hipSetDevice(b->device));
  HIPCHK(hipMemsetAsync(b->db.health, 0, DX_HEALTH_WORDS * 4, b->stream));
  if (b->db.ncon_hist) HIPCHK(hipMemsetAsync(b->db.ncon_hist, 0, DX_NCON_HIST * 4, b->stream));
  return 0;
}

extern "C" int dx_ncon_histogram(dx_batch* b, int enable) {
  if (!b) return fail(DX_EINVAL, "null batch");
  if (enable && !b->ncon_hist) {
    if (int rc = balloc(b, (void**)&b->ncon_hist, DX_NCON_HIST * 4)) return rc;
  }
  b->db.ncon_hist = enable ? b->ncon_hist : nullptr;
  return 0;
}

// ------------------------------------------------------------------------ //
// site Jacobians and batched IK (dx_ik.hip)
// ------------------------------------------------------------------------ //
// Per-call device scratch, released (after the batch stream drains) on every exit path.
struct CallScratch {
  hipStream_t s;
  std::vector<void*> p;
  explicit CallScratch(hipStream_t s_) : s(s_) {}
  ~CallScratch() {
    (void)hipStreamSynchronize(s);
    for (void* q : p) (void)hipFree(q);
  }
  void* get(size_t bytes) {
    void* q = nullptr;
    if (hipMalloc(&q, std::max<size_t>(bytes, 4)) != hipSuccess) return nullptr;
    p.push_back(q);
    return q;
  }
};

static int ik_check_sites(dx_batch* b, const int32_t* sites, int32_t nsite) {
  if (!sites || nsite < 1 || 3 * nsite > 32) return fail(DX_EINVAL, "need 1 <= nsite <= 10 site ids");
  for (int s = 0; s < nsite; s++)
    if (sites[s] < 0 || sites[s] >= b->dm.nsite) return fail(DX_EINVAL, "site id out of range");
  return 0;
}

static int ik_lds_bytes(dx_batch* b, size_t* bytes) {
  *bytes = ((size_t)b->model->lds.total + dx_ik_lds_words(b->dm, 0)) * 4;
  if (*bytes > 160 * 1024) return fail(DX_ELIMIT, "IK LDS footprint exceeds 160 KiB");
  return 0;
}

extern "C" int dx_jac_site(dx_batch* b, const int32_t* sites, int32_t nsite, float* jacp, float* jacr) {
  if (!b) return fail(DX_EINVAL, "null batch");
  if (int rc = ik_check_sites(b, sites, nsite)) return rc;
  size_t lds;
  if (int rc = ik_lds_bytes(b, &lds)) return rc;
  HIPCHK(hipSetDevice(b->device));
  CallScratch S(b->stream);
  IkDev P;
  memset(&P, 0, sizeof(P));
  P.mode = 1;
  P.nsite = nsite;
  P.blk = b->model->lds.total;
  const size_t n = (size_t)b->nenv * 3 * nsite * b->dm.nv;
  int* ds = (int*)S.get(nsite * 4);
  P.jacp = jacp ? (float*)S.get(n * 4) : nullptr;
  P.jacr = jacr ? (float*)S.get(n * 4) : nullptr;
  if (!ds || (jacp && !P.jacp) || (jacr && !P.jacr)) return fail(DX_ENOMEM, "device scratch allocation failed");
  P.sites = ds;
  HIPCHK(hipMemcpyAsync(ds, sites, nsite * 4, hipMemcpyHostToDevice, b->stream));
  HIPCHK(dx_launch_ik(b->nenv, lds, b->stream, b->dm_dev, b->db, b->model->lds, P));
  if (jacp) HIPCHK(hipMemcpyAsync(jacp, P.jacp, n * 4, hipMemcpyDefault, b->stream));
  if (jacr) HIPCHK(hipMemcpyAsync(jacr, P.jacr, n * 4, hipMemcpyDefault, b->stream));
  HIPCHK(hipStreamSynchronize(b->stream));
  return 0;
}

extern "C" int dx_ik_solve(dx_batch* b, const dx_ik_options* opt, const int32_t* sites, int32_t nsite,
                           const int32_t* joints, int32_t njoint, const float* targets, float* qpos_out,
                           int32_t* success, float* linear_err, int32_t* attempt, int32_t* steps) {
  if (!b || !opt || !targets) return fail(DX_EINVAL, "null batch, options or targets");
  if (int rc = ik_check_sites(b, sites, nsite)) return rc;
  if (!joints || njoint < 1 || njoint > DX_MAX_NV) return fail(DX_EINVAL, "need 1 <= njoint <= 64 joint ids");
  const std::vector<int>& jtype = b->model->hi.at("jnt_type");
  for (int k = 0; k < njoint; k++) {
    if (joints[k] < 0 || joints[k] >= b->dm.njnt) return fail(DX_EINVAL, "joint id out of range");
    if (jtype[joints[k]] == DXJ_FREE) return fail(DX_EINVAL, "IK joints must be hinge or slide joints");
  }
  if (opt->max_steps < 1 || opt->num_attempts < 1) return fail(DX_EINVAL, "max_steps and num_attempts must be >= 1");
  if (!(opt->regularization > 0.f)) return fail(DX_EINVAL, "regularization must be positive");
  size_t lds;
  if (int rc = ik_lds_bytes(b, &lds)) return rc;
  const size_t E = b->nenv, A = opt->num_attempts;
  if (E * A > 0x7fffffffull) return fail(DX_EINVAL, "nenv * num_attempts too large");
  HIPCHK(hipSetDevice(b->device));
  CallScratch S(b->stream);
  IkDev P;
  memset(&P, 0, sizeof(P));
  P.mode = 0;
  P.nsite = nsite;
  P.njoint = njoint;
  P.max_steps = opt->max_steps;
  P.early_stop = opt->early_stop != 0;
  P.nattempt = (int)A;
  P.stop_on_first = opt->stop_on_first != 0;
  P.tol = opt->linear_tol;
  P.reg = opt->regularization;
  P.gain = opt->gain;
  P.progress = opt->progress_threshold;
  P.seed = opt->seed;
  P.blk = b->model->lds.total;
  int* ds = (int*)S.get(nsite * 4);
  int* dj = (int*)S.get(njoint * 4);
  float* dt = (float*)S.get(E * 3 * nsite * 4);
  P.att_qpos = (float*)S.get(E * A * njoint * 4);
  P.att_err = (float*)S.get(E * A * nsite * 4);
  P.att_steps = (int*)S.get(E * A * 4);
  float* oq = (float*)S.get(E * njoint * 4);
  int* os = (int*)S.get(E * 4);
  float* oe = (float*)S.get(E * nsite * 4);
  int* oa = (int*)S.get(E * 4);
  int* ot = (int*)S.get(E * 4);
  if (!ds || !dj || !dt || !P.att_qpos || !P.att_err || !P.att_steps || !oq || !os || !oe || !oa || !ot)
    return fail(DX_ENOMEM, "device scratch allocation failed");
  HIPCHK(hipMemcpyAsync(ds, sites, nsite * 4, hipMemcpyHostToDevice, b->stream));
  HIPCHK(hipMemcpyAsync(dj, joints, njoint * 4, hipMemcpyHostToDevice, b->stream));
  HIPCHK(hipMemcpyAsync(dt, targets, E * 3 * nsite * 4, hipMemcpyDefault, b->stream));
  P.sites = ds;
  P.joints = dj;
  P.targets = dt;
  P.starts = nullptr;
  if (A > 1) {  // numpy-compatible random restarts (dx_ik.hip dx_ik_starts_kernel)
    auto it = b->model->arr.find("jnt_range");
    if (it == b->model->arr.end() || it->second.dtype != 1) return fail(DX_EMODEL, "model has no fp64 jnt_range");
    std::vector<double> rng(2 * (size_t)njoint);
    for (int k = 0; k < njoint; k++) {
      rng[2 * k] = ((const double*)it->second.p)[2 * joints[k]];
      rng[2 * k + 1] = ((const double*)it->second.p)[2 * joints[k] + 1];
    }
    double* drng = (double*)S.get(rng.size() * 8);
    uint32_t* mt = (uint32_t*)S.get(E * DX_MT_WORDS * 4);
    float* st = (float*)S.get(E * (A - 1) * njoint * 4);
    if (!drng || !mt || !st) return fail(DX_ENOMEM, "device scratch allocation failed");
    HIPCHK(hipMemcpyAsync(drng, rng.data(), rng.size() * 8, hipMemcpyHostToDevice, b->stream));
    HIPCHK(dx_launch_ik_starts((int)E, (int)A - 1, njoint, opt->seed, drng, mt, st, b->stream));
    P.starts = st;
  }
  HIPCHK(dx_launch_ik((int)(E * A), lds, b->stream, b->dm_dev, b->db, b->model->lds, P));
  HIPCHK(dx_launch_ik_select((int)E, b->stream, b->dm, P, oq, os, oe, oa, ot));
  if (qpos_out) HIPCHK(hipMemcpyAsync(qpos_out, oq, E * njoint * 4, hipMemcpyDefault, b->stream));
  if (success) HIPCHK(hipMemcpyAsync(success, os, E * 4, hipMemcpyDefault, b->stream));
  if (linear_err) HIPCHK(hipMemcpyAsync(linear_err, oe, E * nsite * 4, hipMemcpyDefault, b->stream));
  if (attempt) HIPCHK(hipMemcpyAsync(attempt, oa, E * 4, hipMemcpyDefault, b->stream));
  if (steps) HIPCHK(hipMemcpyAsync(steps, ot, E * 4, hipMemcpyDefault, b->stream));
  HIPCHK(hipStreamSynchronize(b->stream));
  return 0;
}

extern "C" void* dx_stream(dx_batch* b) { return b ? (void*)b->stream : nullptr; }

extern "C" int dx_sync(dx_batch* b) {
  if (!b) return fail(DX_EINVAL, "null batch");
  HIPCHK(hipSetDevice(b->device));
  HIPCHK(hipStreamSynchronize(b->stream));
  return queue_check(b);
}

extern "C" int dx_set_outputs(dx_batch* b, int bodies) {
  if (!b) return fail(DX_EINVAL, "null batch");
  b->db.out_bodies = bodies != 0;
  return 0;
}

extern "C" int dx_sensor_enable(dx_batch* b, int enable) {
  if (!b) return fail(DX_EINVAL, "null batch");
  DevBatch& B = b->db;
  if (enable) {
    if (!b->sen_stash) {
      const size_t E = b->nenv, words = (size_t)b->dm.nq + 2 * b->dm.nv + 1 + 8 * DX_NCON_HI;
      if (int rc = balloc(b, (void**)&b->sen_stash, E * words * 4)) return rc;
      if (int rc = balloc(b, (void**)&b->sensor, E * 3 * b->dm.nbody * 4)) return rc;
    }
    B.sen_stash = b->sen_stash;
  } else {
    B.sen_stash = nullptr;  // buffers stay allocated (and the field readable) until destroy
  }
  return 0;
}

extern "C" int dx_debug_enable(dx_batch* b, int enable) {
  if (!b) return fail(DX_EINVAL, "null batch");
  DevBatch& B = b->db;
  if (enable && !b->debug) {
    size_t E = b->nenv;
    int nv = b->dm.nv;
    int rc = 0;
    rc |= balloc(b, (void**)&B.dbg_qacc_smooth, E * nv * 4);
    rc |= balloc(b, (void**)&B.dbg_qfrc_smooth, E * nv * 4);
    rc |= balloc(b, (void**)&B.dbg_M, E * nv * nv * 4);
    rc |= balloc(b, (void**)&B.dbg_con, E * DX_NCON_HI * 16 * 4);
    rc |= balloc(b, (void**)&B.dbg_nefc, E * 2 * 4);
    if (rc) return rc;
    b->debug = true;
  } else if (!enable) {
    B.dbg_qacc_smooth = nullptr;  // buffers stay allocated until destroy
    B.dbg_qfrc_smooth = nullptr;
    B.dbg_M = nullptr;
    B.dbg_con = nullptr;
    B.dbg_nefc = nullptr;
    b->debug = false;
  }
  return 0;
}

extern "C" int dx_debug_get(dx_batch* b, const char* name, float* dst, size_t nfloats) {
  if (!b || !name || !dst) return fail(DX_EINVAL, "null argument");
  DevBatch& B = b->db;
  if (std::string(name) == "queue_timeouts") {  // int32 bits: 1 if a queued task ever gave up waiting
    if (nfloats < 1) return fail(DX_EINVAL, "destination too small");
    HIPCHK(hipSetDevice(b->device));
    HIPCHK(hipMemcpyAsync(dst, B.qerr, 4, hipMemcpyDeviceToHost, b->stream));
    HIPCHK(hipStreamSynchronize(b->stream));
    return 0;
  }
  if (std::string(name) == "health") {  // uint32 bits: dx_health's counters (+ histogram)
    return dx_health(b, (uint32_t*)dst, (int32_t)std::min<size_t>(nfloats, DX_HEALTH_WORDS + DX_NCON_HIST));
  }
  if (std::string(name) == "queue_slots") {  // int32 bits: the queued launch's persistent workgroups
    if (nfloats < 1) return fail(DX_EINVAL, "destination too small");
    memcpy(dst, &b->slots, 4);
    return 0;
  }
  if (!b->debug) return fail(DX_EINVAL, "debug not enabled");
  size_t E = b->nenv, nv = b->dm.nv;
  const void* src = nullptr;
  size_t n = 0;
  std::string s(name);
  if (s == "qacc_smooth") { src = B.dbg_qacc_smooth; n = E * nv; }
  else if (s == "qfrc_smooth") { src = B.dbg_qfrc_smooth; n = E * nv; }
  else if (s == "M") { src = B.dbg_M; n = E * nv * nv; }
  else if (s == "contact") { src = B.dbg_con; n = E * DX_NCON_HI * 16; }
  else if (s == "efc_count") { src = B.dbg_nefc; n = E * 2; }
  else return fail(DX_EINVAL, "unknown debug field");
  if (nfloats < n) return fail(DX_EINVAL, "destination too small");
  HIPCHK(hipSetDevice(b->device));
  HIPCHK(hipMemcpyAsync(dst, src, n * 4, hipMemcpyDeviceToHost, b->stream));
  HIPCHK(hipStreamSynchronize(b->stream));
  return 0;
}

// ------------------------------------------------------------------------ //
// environments: physics batch + on-device task logic
// ------------------------------------------------------------------------ //
extern "C" __global__ void dx_task_pre_kernel(TaskParams P, TaskState S, DevBatch B, const float* qpos0,
                                              const float* action);
extern "C" __global__ void dx_task_post_kernel(TaskParams P, TaskState S, DevBatch B);
extern "C" __global__ void dx_mt_seed_kernel(int nenv, uint64_t seed, uint32_t* mt_env, uint32_t* mt_goal);
extern "C" __global__ void dx_mtw_seed_kernel(int nenv, uint64_t seed, uint32_t* mt);

struct dx_env {
  dx_batch* batch;
  TaskParams P;
  TaskState S;
  int nsub;
  std::vector<void*> allocs;
};

extern "C" dx_env* dx_env_create(const dx_model* m, int32_t nenv, int32_t device, int32_t task,
                                 uint64_t seed, const float* params, int32_t nparams) {
  return dx_env_create_shard(m, nenv, device, task, seed, 0, params, nparams);
}

extern "C" dx_env* dx_env_create_shard(const dx_model* m, int32_t nenv, int32_t device, int32_t task,
                                       uint64_t seed, int64_t env0, const float* params, int32_t nparams) {
  if (env0 < 0 || env0 + (int64_t)nenv > 0x7fffffffll) { fail(DX_EINVAL, "env0 out of range"); return nullptr; }
  if (task != DX_TASK_REORIENT && task != DX_TASK_REACH && task != DX_TASK_HANDOVER) {
    fail(DX_EINVAL, "unknown task kind");
    return nullptr;
  }
  if (!m) { fail(DX_EINVAL, "null model"); return nullptr; }
  const int nq = m->dm.nq, nu = m->dm.nu;
  if (!params || (task == DX_TASK_REORIENT && nparams < DX_REORIENT_NPARAMS) ||
      (task == DX_TASK_HANDOVER && nparams < DX_HANDOVER_NPARAMS) ||
      (task == DX_TASK_REACH && nparams < DX_REACH_NPARAMS_HEAD + 3 * nq + nu * nq)) {
    fail(DX_EINVAL, "too few task params");
    return nullptr;
  }
  dx_batch* b = dx_batch_create(m, nenv, device);
  if (!b) return nullptr;
  dx_env* e = new dx_env();
  e->batch = b;
  const DevModel& d = b->dm;
  TaskParams& P = e->P;
  memset(&P, 0, sizeof(P));
  P.kind = task == DX_TASK_REACH ? DX_KIND_REACH : task == DX_TASK_HANDOVER ? DX_KIND_HANDOVER : DX_KIND_REORIENT;
  P.nenv = nenv; P.nq = d.nq; P.nv = d.nv; P.nu = d.nu; P.nsite = d.nsite;
  P.seed = seed;
  P.env0 = (int)env0;
  e->nsub = (int)params[0];
  P.hand_nq = (int)params[1]; P.hand_nv = (int)params[2];
  int watch_geom = -1, watch_body = -1;
  bool bad = false;
  if (task != DX_TASK_REACH) {  // reorient, and the handover on the same params
    P.prop_qadr = (int)params[3]; P.prop_dadr = (int)params[4];
    int tip0 = (int)params[5];
    P.ntips = (int)params[6];
    for (int t = 0; t < P.ntips && t < DX_MAX_TIPS; t++) P.tip_sites[t] = tip0 + t;
    P.successes_needed = (int)params[7]; P.steps_before_change = (int)params[8];
    P.fall_termination = (int)params[9];
    P.threshold = params[10]; P.eps = params[11]; P.w_orient = params[12]; P.w_success = params[13];
    P.w_action = params[14]; P.max_time = params[15];
    for (int k = 0; k < 3; k++) {
      P.bbox_lo[k] = params[16 + k]; P.bbox_hi[k] = params[19 + k];
      // fp64 box: the raw bits of six doubles in params 26-37, when given
      P.bbox_lo_d[k] = params[16 + k];
      P.bbox_hi_d[k] = params[19 + k];
      if (nparams >= 38) {
        memcpy(&P.bbox_lo_d[k], params + 26 + 2 * k, 8);
        memcpy(&P.bbox_hi_d[k], params + 32 + 2 * k, 8);
      }
    }
    watch_geom = (int)params[22]; watch_body = (int)params[23];
    P.goal_dim = 4;  // the target quaternion, or (handover) the target point and receiving hand
    // (the handover has no hint prop: no target_prop/orientation block)
    const int prop_obs = P.prop_qadr < 0 ? 0 : task == DX_TASK_HANDOVER ? 13 : 17;
    P.obs_dim = 2 * P.hand_nq + P.hand_nv + 6 * P.ntips + prop_obs + 4;
    bad = P.prop_qadr >= 0 && (P.prop_qadr + 7 > d.nq || P.prop_dadr + 6 > d.nv);
    if (task == DX_TASK_HANDOVER) {
      for (int h = 0; h < 2; h++)
        for (int k = 0; k < 3; k++) P.hand_target[h][k] = params[38 + 3 * h + k];
      bad = bad || P.prop_qadr < 0;
    }
  } else {
    P.prop_qadr = -1; P.prop_dadr = -1;
    P.ntips = (int)params[3];
    for (int t = 0; t < P.ntips && t < DX_MAX_TIPS; t++) P.tip_sites[t] = (int)params[4 + t];
    P.successes_needed = (int)params[9]; P.steps_before_change = (int)params[10];
    P.threshold = params[11]; P.max_time = params[12]; P.dense = (int)params[13];
    P.range_frac = params[14]; P.goal_scale = params[15]; P.max_reject = (int)params[16];
    P.ncoupled = (int)params[17];
    for (int k = 0; k < P.ncoupled && k < 4; k++) {
      P.coupled[k][0] = (int)params[18 + 2 * k];
      P.coupled[k][1] = (int)params[19 + 2 * k];
      bad = bad || P.coupled[k][0] < 0 || P.coupled[k][0] >= nq || P.coupled[k][1] < 0 || P.coupled[k][1] >= nq;
    }
    P.goal_dim = 3 * P.ntips;
    P.obs_dim = 2 * P.hand_nq + P.hand_nv + 6 * P.ntips + P.goal_dim;
    bad = bad || P.hand_nq != d.nq || P.ncoupled > 4 || P.max_reject < 1;
  }
  for (int t = 0; t < P.ntips && t < DX_MAX_TIPS; t++) bad = bad || P.tip_sites[t] < 0 || P.tip_sites[t] >= d.nsite;
  if (bad || P.ntips > DX_MAX_TIPS || P.hand_nq > d.nq || P.hand_nv > d.nv || e->nsub < 1) {
    fail(DX_EINVAL, "task parameters inconsistent with the model");
    dx_batch_destroy(b);
    delete e;
    return nullptr;
  }
  if (watch_geom >= 0 && dx_set_watch(b, watch_geom, watch_body) != 0) { dx_batch_destroy(b); delete e; return nullptr; }
  TaskState& S = e->S;
  size_t E = nenv;
  auto al = [&](void** p, size_t bytes) { return balloc(b, p, bytes); };
  int rc = 0;
  rc |= al((void**)&S.goal, E * P.goal_dim * 4); rc |= al((void**)&S.solve_start, E * 4);
  rc |= al((void**)&S.reward, E * 4); rc |= al((void**)&S.discount, E * 4);
  rc |= al((void**)&S.obs, E * P.obs_dim * 4);
  rc |= al((void**)&S.successes, E * 4); rc |= al((void**)&S.counter, E * 4);
  rc |= al((void**)&S.registered, E * 4); rc |= al((void**)&S.exceeded, E * 4);
  rc |= al((void**)&S.step_type, E * 4); rc |= al((void**)&S.episode, E * 4);
  rc |= al((void**)&S.skip, E * 4); rc |= al((void**)&S.failure, E * 4);
  rc |= al((void**)&S.need, E * 4); rc |= al((void**)&S.goalnum, E * 4); rc |= al((void**)&S.goalfail, E * 4);
  rc |= al((void**)&S.time_d, E * 8); rc |= al((void**)&S.solve_start_d, E * 8);
  rc |= al((void**)&S.nsub_d, E * 4); rc |= al((void**)&S.solve_n, E * 4);
  if (task == DX_TASK_REACH) rc |= al((void**)&S.goal_qpos, E * nq * 4);
  if (task != DX_TASK_REACH) {
    rc |= al((void**)&S.mt_env, E * DX_MT_WORDS * 4);
    rc |= al((void**)&S.mt_goal, E * DX_MT_WORDS * 4);
    if (!rc) {
      hipLaunchKernelGGL(dx_mt_seed_kernel, dim3((nenv + 63) / 64), dim3(64), 0, b->stream, nenv, seed + (uint64_t)env0, S.mt_env,
                         S.mt_goal);
      if (hipGetLastError() != hipSuccess) rc = fail(DX_EHIP, "MT19937 seeding kernel launch failed");
    }
  }
  P.time_limit = INFINITY;
  P.time_limit_d = INFINITY;
  P.h_d = getd(m, "timestep");
  P.max_time_d = P.max_time;  // dx_env_set_goal_time_limit gives the fp64 value
  float* tdata = nullptr;
  TaskParams* dP = nullptr;
  TaskState* dS = nullptr;
  if (!rc && task == DX_TASK_REACH) {
    size_t nt = 3 * (size_t)nq + (size_t)nu * nq;
    // optional fp64 block (raw bits of 6 x nq doubles) for numpy-compatible draws
    if (nparams >= DX_REACH_NPARAMS_HEAD + (int)nt + 12 * nq) {
      nt += 12 * (size_t)nq;
      P.tdata_f64 = 1;
      rc |= al((void**)&S.mt_reach, E * DX_MTW_WORDS * 4);
      if (!rc) {
        hipLaunchKernelGGL(dx_mtw_seed_kernel, dim3((nenv + 63) / 64), dim3(64), 0, b->stream, nenv,
                           seed + (uint64_t)env0, S.mt_reach);
        if (hipGetLastError() != hipSuccess) rc = fail(DX_EHIP, "MT19937 seeding kernel launch failed");
      }
    }
    rc |= al((void**)&tdata, nt * 4);
    // balloc zeroes on the batch's (non-blocking) stream: drain it before the
    // synchronous copies below, or a late memset can wipe what they wrote
    if (!rc && hipStreamSynchronize(b->stream) != hipSuccess) rc = fail(DX_EHIP, "stream sync failed");
    if (!rc && hipMemcpy(tdata, params + DX_REACH_NPARAMS_HEAD, nt * 4, hipMemcpyHostToDevice) != hipSuccess)
      rc = fail(DX_EHIP, "hipMemcpy failed");
    P.tdata = tdata;
  }
  if (!rc) rc |= al((void**)&dP, sizeof(TaskParams));
  if (!rc) rc |= al((void**)&dS, sizeof(TaskState));
  std::vector<int> neg(E, -1);
  if (!rc && hipStreamSynchronize(b->stream) != hipSuccess) rc = fail(DX_EHIP, "stream sync failed");
  if (!rc && (hipMemcpy(S.episode, neg.data(), E * 4, hipMemcpyHostToDevice) != hipSuccess ||
              hipMemcpy(dP, &P, sizeof(P), hipMemcpyHostToDevice) != hipSuccess ||
              hipMemcpy(dS, &S, sizeof(S), hipMemcpyHostToDevice) != hipSuccess))
    rc = fail(DX_EHIP, "hipMemcpy failed");
  if (rc) { dx_batch_destroy(b); delete e; return nullptr; }
  b->db.skip = S.skip;
  b->db.out_bodies = 0;  // the tasks read sites and qpos only (dx_set_outputs turns body poses back on)
  b->db.tp = dP;
  b->db.ts = dS;
  return e;
}

extern "C" int dx_env_goal_dim(const dx_env* e) { return e ? e->P.goal_dim : fail(DX_EINVAL, "null env"); }

extern "C" void dx_env_destroy(dx_env* e) {
  if (!e) return;
  dx_batch_destroy(e->batch);
  delete e;
}

extern "C" dx_batch* dx_env_batch(dx_env* e) { return e ? e->batch : nullptr; }
extern "C" int dx_env_obs_dim(const dx_env* e) { return e ? e->P.obs_dim : fail(DX_EINVAL, "null env"); }

extern "C" __global__ void dx_sample_actions_kernel(int nenv, int nu, const float* ctrlrange, uint64_t seed,
                                                    int step, int env0, float* out);

// One control step.  The task logic runs fused into the step kernel (task_pre in each
// env's first physics-step task, task_post in its last; dx_task.h): a reorient control step
// is the step kernel plus the overflow tier's launch.  Reach (a reach scene's
// specialization) also runs its sampling pass -- goal rollouts, joint sampling -- in the
// env's first task (dx_step.hip fused_reach_prep): the step kernel plus the order kernel
// (contact-free Shadow reach) or the overflow tier (Adroit).  DX_NO_FUSE=1 selects the
// task kernels and the separate sampling launch instead.
// random: actions drawn in the kernel by the random agent (seed, step) instead of read.
static int env_run(dx_env* e, const float* action, bool random = false, uint64_t seed = 0, int step = 0) {
  dx_batch* b = e->batch;
  HIPCHK(hipSetDevice(b->device));
  const bool fuse = !getenv("DX_NO_FUSE") && ((e->P.kind != DX_KIND_REACH && b->db.defer) ||
                                              (e->P.kind == DX_KIND_REACH && b->spec >= 0 && dx_spec_reach(b->spec)));
  if (fuse) {
    DevBatch& B = b->db;
    const int* skip = B.skip;
    B.fuse = 1;
    B.skip = nullptr;
    B.action = action;
    B.act_random = random ? 1 : 0;
    B.act_seed = seed;
    B.act_step = step;
    const int rc = launch_step(b, e->nsub, 0);
    B.fuse = 0;
    B.skip = skip;
    B.action = nullptr;
    B.act_random = 0;
    return rc;
  }
  if (random) {  // the random agent into the action buffer, then the step
    void* buf = nullptr;
    if (int rc = dx_env_action_buffer(e, &buf)) return rc;
    hipLaunchKernelGGL(dx_sample_actions_kernel, dim3((e->P.nenv * e->P.nu + 255) / 256), dim3(256), 0, b->stream,
                       e->P.nenv, e->P.nu, b->dm.actuator_ctrlrange, seed, step, e->P.env0, (float*)buf);
    HIPCHK(hipGetLastError());
    action = (const float*)buf;
  }
  int nb = (e->P.nenv + 63) / 64;
  hipLaunchKernelGGL(dx_task_pre_kernel, dim3(nb), dim3(64), 0, b->stream, e->P, e->S, b->db,
                     b->dm.qpos0, action);
  HIPCHK(hipGetLastError());
  // reach: goal rollouts / joint sampling for the envs that need them (the rest of
  // the grid exits at once)
  if (e->P.kind == DX_KIND_REACH)
    if (int rc = launch_step(b, 1, 2)) return rc;
  if (int rc = launch_step(b, e->nsub, 0)) return rc;
  hipLaunchKernelGGL(dx_task_post_kernel, dim3((e->P.nenv + 3) / 4), dim3(256), 0, b->stream, e->P, e->S, b->db);  // a wave per env
  HIPCHK(hipGetLastError());
  return 0;
}

extern "C" int dx_env_reset(dx_env* e) {
  if (!e) return fail(DX_EINVAL, "null env");
  // step_type LAST makes the pre-kernel run initialize_episode for every env
  std::vector<int> last(e->P.nenv, 2);
  HIPCHK(hipMemcpyAsync(e->S.step_type, last.data(), last.size() * 4, hipMemcpyHostToDevice, e->batch->stream));
  HIPCHK(hipStreamSynchronize(e->batch->stream));
  return env_run(e, nullptr);
}

static int env_params_upload(dx_env* e) {
  HIPCHK(hipSetDevice(e->batch->device));
  HIPCHK(hipStreamSynchronize(e->batch->stream));  // the device copy is read by the sampling pass
  HIPCHK(hipMemcpy((void*)e->batch->db.tp, &e->P, sizeof(TaskParams), hipMemcpyHostToDevice));
  return 0;
}

extern "C" int dx_env_set_time_limit(dx_env* e, double seconds) {
  if (!e || !(seconds > 0)) return fail(DX_EINVAL, "null env or non-positive time limit");
  e->P.time_limit = (float)seconds;
  e->P.time_limit_d = seconds;
  return env_params_upload(e);
}

extern "C" int dx_env_set_goal_time_limit(dx_env* e, double seconds) {
  if (!e || !(seconds >= 0)) return fail(DX_EINVAL, "null env or negative time");
  e->P.max_time = (float)seconds;
  e->P.max_time_d = seconds;
  return env_params_upload(e);
}

extern "C" int dx_env_step(dx_env* e, const float* action) {
  if (!e || !action) return fail(DX_EINVAL, "null env or action");
  return env_run(e, action);
}

extern "C" int dx_env_step_random(dx_env* e, uint64_t seed, int32_t step) {
  if (!e) return fail(DX_EINVAL, "null env");
  return env_run(e, nullptr, true, seed, step);
}

// ------------------------------------------------------------------------ //
// checkpoint / resume: every device array whose contents carry from one
// control step to the next -- physics state (qpos, qvel, ctrl, warm start, fp32 time, the
// physics-step count behind the fp64 time), task state (goals, counters, step types, fp64
// times, observation, rewards), both numpy-compatible MT19937 streams of an env (reach:
// the RandomState block with numpy's cached gaussian), and the longest-first order.  The
// separating-direction cache is left out: it never changes a result (dx_step.hip
// mpr_init).  Restoring into an env of the same task, model and size resumes the run bit
// for bit.
// ------------------------------------------------------------------------ //
struct StateField {
  const char* name;
  void* ptr;
  size_t bytes;
};
static std::vector<StateField> env_state_fields(dx_env* e) {
  dx_batch* b = e->batch;
  const DevBatch& B = b->db;
  const TaskState& S = e->S;
  const TaskParams& P = e->P;
  const size_t E = b->nenv;
  const DevModel& d = b->dm;
  std::vector<StateField> f = {
      {"qpos", B.qpos, E * d.nq * 4}, {"qvel", B.qvel, E * d.nv * 4},
      {"ctrl", B.ctrl, E * std::max(d.nu, 1) * 4}, {"qacc_warmstart", B.qacc_ws, E * d.nv * 4},
      {"qacc", B.qacc, E * d.nv * 4}, {"time", B.time, E * 4}, {"nstep", B.nstep, E * 4},
      {"diverged", B.bad, E * 4},
      {"goal", S.goal, E * P.goal_dim * 4}, {"solve_start", S.solve_start, E * 4},
      {"reward", S.reward, E * 4}, {"discount", S.discount, E * 4}, {"obs", S.obs, E * P.obs_dim * 4},
      {"successes", S.successes, E * 4}, {"counter", S.counter, E * 4}, {"registered", S.registered, E * 4},
      {"exceeded", S.exceeded, E * 4}, {"step_type", S.step_type, E * 4}, {"episode", S.episode, E * 4},
      {"skip", S.skip, E * 4}, {"failure", S.failure, E * 4}, {"need", S.need, E * 4},
      {"goalnum", S.goalnum, E * 4}, {"goalfail", S.goalfail, E * 4}, {"time_d", S.time_d, E * 8},
      {"solve_start_d", S.solve_start_d, E * 8}, {"nsub_d", S.nsub_d, E * 4}, {"solve_n", S.solve_n, E * 4},
  };
  if (S.goal_qpos) f.push_back({"goal_qpos", S.goal_qpos, E * d.nq * 4});
  if (S.mt_env) f.push_back({"mt_env", S.mt_env, E * DX_MT_WORDS * 4});
  if (S.mt_goal) f.push_back({"mt_goal", S.mt_goal, E * DX_MT_WORDS * 4});
  if (S.mt_reach) f.push_back({"mt_reach", S.mt_reach, E * DX_MTW_WORDS * 4});
  if (B.cost) f.push_back({"step_cost", B.cost, E * 4});
  if (B.order) f.push_back({"order", (void*)B.order, E * 4});
  return f;
}

extern "C" int dx_env_state_field(dx_env* e, int32_t i, const char** name, size_t* offset, size_t* nbytes) {
  if (!e || !name || !offset || !nbytes) return fail(DX_EINVAL, "null argument");
  const auto f = env_state_fields(e);
  if (i < 0) return (int)f.size();
  if (i >= (int)f.size()) return fail(DX_EINVAL, "state field out of range");
  size_t off = 0;
  for (int k = 0; k < i; k++) off += f[k].bytes;
  *name = f[i].name;
  *offset = off;
  *nbytes = f[i].bytes;
  return (int)f.size();
}

extern "C" int dx_env_save(dx_env* e, void* dst, size_t nbytes) {
  if (!e) return fail(DX_EINVAL, "null env");
  const auto f = env_state_fields(e);
  size_t tot = 0;
  for (auto& x : f) tot += x.bytes;
  if (!dst) return (int)std::min<size_t>(tot, 0x7fffffff);  // the size query
  if (nbytes < tot) return fail(DX_EINVAL, "checkpoint buffer too small");
  dx_batch* b = e->batch;
  HIPCHK(hipSetDevice(b->device));
  size_t off = 0;
  for (auto& x : f) {
    HIPCHK(hipMemcpyAsync((char*)dst + off, x.ptr, x.bytes, hipMemcpyDefault, b->stream));
    off += x.bytes;
  }
  HIPCHK(hipStreamSynchronize(b->stream));
  return queue_check(b);
}

extern "C" int dx_env_load(dx_env* e, const void* src, size_t nbytes) {
  if (!e || !src) return fail(DX_EINVAL, "null argument");
  const auto f = env_state_fields(e);
  size_t tot = 0;
  for (auto& x : f) tot += x.bytes;
  if (nbytes != tot) return fail(DX_EINVAL, "checkpoint size does not match this env (task, model, batch size)");
  dx_batch* b = e->batch;
  HIPCHK(hipSetDevice(b->device));
  size_t off = 0;
  for (auto& x : f) {
    HIPCHK(hipMemcpyAsync(x.ptr, (const char*)src + off, x.bytes, hipMemcpyDefault, b->stream));
    off += x.bytes;
  }
  HIPCHK(hipStreamSynchronize(b->stream));
  return 0;
}

extern "C" int dx_env_output(dx_env* e, int which, void** devptr) {
  if (!e || !devptr) return fail(DX_EINVAL, "null argument");
  switch (which) {
    case DX_OUT_OBS: *devptr = e->S.obs; return 0;
    case DX_OUT_REWARD: *devptr = e->S.reward; return 0;
    case DX_OUT_DISCOUNT: *devptr = e->S.discount; return 0;
    case DX_OUT_STEP_TYPE: *devptr = e->S.step_type; return 0;
    case DX_OUT_GOAL: *devptr = e->S.goal; return 0;
    case DX_OUT_SUCCESSES: *devptr = e->S.successes; return 0;
    case DX_OUT_GOAL_FAILURES: *devptr = e->S.goalfail; return 0;
    case DX_OUT_GOAL_QPOS:
      if (!e->S.goal_qpos) return fail(DX_EINVAL, "goal joints exist for the reach task only");
      *devptr = e->S.goal_qpos;
      return 0;
  }
  return fail(DX_EINVAL, "unknown output");
}

extern "C" int dx_env_action_buffer(dx_env* e, void** devptr) {
  if (!e || !devptr) return fail(DX_EINVAL, "null argument");
  if (e->allocs.empty()) {
    void* p = nullptr;
    if (int rc = balloc(e->batch, &p, (size_t)e->P.nenv * std::max(e->P.nu, 1) * 4)) return rc;
    e->allocs.push_back(p);
  }
  *devptr = e->allocs[0];
  return 0;
}

extern "C" int dx_env_sample_actions(dx_env* e, uint64_t seed, int32_t step) {
  if (!e) return fail(DX_EINVAL, "null env");
  void* buf = nullptr;
  if (int rc = dx_env_action_buffer(e, &buf)) return rc;
  dx_batch* b = e->batch;
  HIPCHK(hipSetDevice(b->device));
  int n = e->P.nenv * e->P.nu;
  hipLaunchKernelGGL(dx_sample_actions_kernel, dim3((n + 255) / 256), dim3(256), 0, b->stream, e->P.nenv,
                     e->P.nu, b->dm.actuator_ctrlrange, seed, step, e->P.env0, (float*)buf);
  HIPCHK(hipGetLastError());
  return 0;
}

// ------------------------------------------------------------------------ //
// kernel timing (HIP events around every step-kernel launch on the batch stream)
// ------------------------------------------------------------------------ //
struct TimingState {
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev;
  bool on = false;
  unsigned n = 0, every = 1;
};
static std::map<const dx_batch*, TimingState> g_timing;

static void timing_begin(dx_batch* b, hipEvent_t* start) {
  auto it = g_timing.find(b);
  *start = nullptr;
  if (it == g_timing.end() || !it->second.on) return;
  if (it->second.n++ % it->second.every) return;  // (every every-th launch, dx_timing_enable)
  (void)hipEventCreate(start);
  (void)hipEventRecord(*start, b->stream);
}
static void timing_end(dx_batch* b, hipEvent_t start) {
  if (!start) return;
  hipEvent_t stop;
  (void)hipEventCreate(&stop);
  (void)hipEventRecord(stop, b->stream);
  g_timing[b].ev.emplace_back(start, stop);
}

extern "C" int dx_timing_enable(dx_batch* b, int enable) {
  if (!b) return fail(DX_EINVAL, "null batch");
  auto& st = g_timing[b];
  st.on = enable != 0;
  st.every = (unsigned)std::max(1, enable);
  st.n = 0;
  return 0;
}

extern "C" int dx_timing_read(dx_batch* b, double* total_ms, int32_t* count) {
  if (!b || !total_ms || !count) return fail(DX_EINVAL, "null argument");
  HIPCHK(hipSetDevice(b->device));
  HIPCHK(hipStreamSynchronize(b->stream));
  double tot = 0;
  auto& st = g_timing[b];
  for (auto& p : st.ev) {
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, p.first, p.second));
    tot += ms;
    (void)hipEventDestroy(p.first);
    (void)hipEventDestroy(p.second);
  }
  *total_ms = tot;
  *count = (int32_t)st.ev.size();
  st.ev.clear();
  return queue_check(b);
}

// packs [obs | reward | discount | step_type] per env into dst (device, [nenv][obs_dim+3])
extern "C" __global__ void dx_pack_outputs_kernel(int nenv, int obs_dim, const float* obs, const float* rew,
                                                  const float* disc, const int* st, float* dst);

extern "C" int dx_env_pack_outputs(dx_env* e, float* dst_dev) {
  if (!e || !dst_dev) return fail(DX_EINVAL, "null argument");
  dx_batch* b = e->batch;
  HIPCHK(hipSetDevice(b->device));
  int n = e->P.nenv * (e->P.obs_dim + 3);
  hipLaunchKernelGGL(dx_pack_outputs_kernel, dim3((n + 255) / 256), dim3(256), 0, b->stream, e->P.nenv,
                     e->P.obs_dim, e->S.obs, e->S.reward, e->S.discount, e->S.step_type, dst_dev);
  HIPCHK(hipGetLastError());
  return 0;
}

#ifndef DX_BUILD_KEY
#define DX_BUILD_KEY "unkeyed"
#endif
// The hash of the sources this library was built from (dexterity_amd/build.py source_key)
extern "C" const char* dx_build_key(void) { return DX_BUILD_KEY; }

// The reference's own call shape: GoalEnvironment.step(action) with a host action and a
// host TimeStep back (environment.py:25-34, task.py:63-73).  One stream: the action's
// upload into the library's action buffer, the control step, the pack of [obs | reward |
// discount | step_type] and its download, then one synchronisation.  With page-locked
// host buffers both copies are DMA transfers queued behind / ahead of the kernels.
extern "C" int dx_env_step_host(dx_env* e, const float* action_host, float* out_host) {
  if (!e || !action_host || !out_host) return fail(DX_EINVAL, "null argument");
  dx_batch* b = e->batch;
  HIPCHK(hipSetDevice(b->device));
  void* act = nullptr;
  if (int rc = dx_env_action_buffer(e, &act)) return rc;
  const size_t nout = (size_t)e->P.nenv * (e->P.obs_dim + 3);
  if (e->allocs.size() < 2) {  // the packed outputs' device buffer
    void* p = nullptr;
    if (int rc = balloc(b, &p, nout * 4)) return rc;
    e->allocs.push_back(p);
  }
  float* pack = (float*)e->allocs[1];
  HIPCHK(hipMemcpyAsync(act, action_host, (size_t)e->P.nenv * e->P.nu * 4, hipMemcpyHostToDevice, b->stream));
  if (int rc = env_run(e, (const float*)act)) return rc;
  if (int rc = dx_env_pack_outputs(e, pack)) return rc;
  HIPCHK(hipMemcpyAsync(out_host, pack, nout * 4, hipMemcpyDeviceToHost, b->stream));
  HIPCHK(hipStreamSynchronize(b->stream));
  return 0;
}

// ------------------------------------------------------------------------ //
// multi-GPU observation collation: RCCL (librccl) directly, no framework layer
// ------------------------------------------------------------------------ //
// One process per GPU.  Physics has no exchange (environments are independent);
// the only collective is the per-control-step all-gather of the packed outputs,
// enqueued on the env's stream right behind the task post kernel, so the host
// never waits for it.  The gather is in place: this rank packs straight into its
// own slice of dst.
struct dx_comm {
  ncclComm_t comm = nullptr;
  int rank = 0, nranks = 1, device = 0;
  hipStream_t stream = nullptr;  // barrier / scalar reductions
  double* scalar = nullptr;      // device scratch for dx_comm_allreduce_max
};

#define NCCLCHK(x)                                                                                 \
  do {                                                                                             \
    ncclResult_t r_ = (x);                                                                         \
    if (r_ != ncclSuccess) return fail(DX_EHIP, std::string(#x ": ") + ncclGetErrorString(r_));    \
  } while (0)

extern "C" int dx_comm_unique_id(void* id) {
  if (!id) return fail(DX_EINVAL, "null id buffer");
  static_assert(sizeof(ncclUniqueId) == DX_COMM_ID_BYTES, "RCCL unique id size");
  ncclUniqueId u;
  NCCLCHK(ncclGetUniqueId(&u));
  memcpy(id, &u, sizeof(u));
  return 0;
}

extern "C" dx_comm* dx_comm_init(const void* id, int32_t nranks, int32_t rank, int32_t device) {
  if (!id || nranks < 1 || rank < 0 || rank >= nranks) { fail(DX_EINVAL, "bad comm arguments"); return nullptr; }
  if (hipSetDevice(device) != hipSuccess) { fail(DX_EHIP, "hipSetDevice failed"); return nullptr; }
  dx_comm* c = new dx_comm();
  c->rank = rank;
  c->nranks = nranks;
  c->device = device;
  ncclUniqueId u;
  memcpy(&u, id, sizeof(u));
  ncclResult_t r = ncclCommInitRank(&c->comm, nranks, u, rank);
  if (r != ncclSuccess) {
    fail(DX_EHIP, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
    delete c;
    return nullptr;
  }
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipMalloc(&c->scalar, sizeof(double)) != hipSuccess) {
    fail(DX_EHIP, "comm stream / scratch allocation failed");
    dx_comm_destroy(c);
    return nullptr;
  }
  return c;
}

extern "C" void dx_comm_destroy(dx_comm* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->comm) (void)ncclCommDestroy(c->comm);
  if (c->scalar) (void)hipFree(c->scalar);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

extern "C" int dx_comm_rank(const dx_comm* c) { return c ? c->rank : fail(DX_EINVAL, "null comm"); }
extern "C" int dx_comm_size(const dx_comm* c) { return c ? c->nranks : fail(DX_EINVAL, "null comm"); }

extern "C" int dx_allgather_obs(dx_env* e, dx_comm* c, float* dst_dev) {
  if (!e || !c || !dst_dev) return fail(DX_EINVAL, "null argument");
  dx_batch* b = e->batch;
  if (b->device != c->device) return fail(DX_EINVAL, "env and comm are on different devices");
  const size_t count = (size_t)e->P.nenv * (e->P.obs_dim + 3);
  float* mine = dst_dev + (size_t)c->rank * count;
  if (int rc = dx_env_pack_outputs(e, mine)) return rc;
  NCCLCHK(ncclAllGather(mine, dst_dev, count, ncclFloat32, c->comm, b->stream));
  return 0;
}

extern "C" int dx_comm_allreduce_max(dx_comm* c, double* value) {
  if (!c || !value) return fail(DX_EINVAL, "null argument");
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipMemcpyAsync(c->scalar, value, sizeof(double), hipMemcpyHostToDevice, c->stream));
  NCCLCHK(ncclAllReduce(c->scalar, c->scalar, 1, ncclFloat64, ncclMax, c->comm, c->stream));
  HIPCHK(hipMemcpyAsync(value, c->scalar, sizeof(double), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

extern "C" int dx_comm_barrier(dx_comm* c) {
  double x = 0;
  return dx_comm_allreduce_max(c, &x);
}

// Fills every CU's LDS with NaN bit patterns (test hook: the step kernel must not
// depend on LDS contents left by earlier workgroups).
__global__ void dx_poison_lds_kernel(int nwords) {
  extern __shared__ unsigned int lds_words[];
  for (int k = threadIdx.x; k < nwords; k += blockDim.x) lds_words[k] = 0x7fc00000u | (k & 0xff);
  __syncthreads();
}

extern "C" int dx_debug_poison_lds(int32_t device) {
  HIPCHK(hipSetDevice(device));
  const int bytes = 64 * 1024;
  hipLaunchKernelGGL(dx_poison_lds_kernel, dim3(256 * 16), dim3(256), bytes, nullptr, bytes / 4);
  HIPCHK(hipGetLastError());
  HIPCHK(hipDeviceSynchronize());
  return 0;
}

extern "C" int dx_stage_timing(dx_batch* b, int enable) {
  if (!b) return fail(DX_EINVAL, "null batch");
  HIPCHK(hipSetDevice(b->device));
  size_t bytes = (size_t)b->nenv * DX_NSTAGE * 8;  // per-env accumulators: no atomics
  if (enable && !b->db.stage_acc) {
    void* p = nullptr;
    if (int rc = balloc(b, &p, bytes)) return rc;
    HIPCHK(hipMemsetAsync(p, 0, bytes, b->stream));
    b->db.stage_acc = (unsigned long long*)p;
  } else if (!enable) {
    b->db.stage_acc = nullptr;
  }
  return 0;
}

extern "C" int dx_stage_read(dx_batch* b, uint64_t* out, int32_t n) {
  if (!b || !out) return fail(DX_EINVAL, "null argument");
  if (!b->db.stage_acc) return fail(DX_EINVAL, "stage timing not enabled");
  HIPCHK(hipSetDevice(b->device));
  size_t cnt = (size_t)b->nenv * DX_NSTAGE;
  std::vector<uint64_t> h(cnt);
  HIPCHK(hipMemcpyAsync(h.data(), b->db.stage_acc, cnt * 8, hipMemcpyDeviceToHost, b->stream));
  HIPCHK(hipMemsetAsync(b->db.stage_acc, 0, cnt * 8, b->stream));
  HIPCHK(hipStreamSynchronize(b->stream));
  if ((size_t)n >= cnt) {  // per env: out[env][DX_NSTAGE]
    memcpy(out, h.data(), cnt * 8);
    return 0;
  }
  for (int k = 0; k < std::min(n, DX_NSTAGE); k++) {
    uint64_t t = 0;
    for (int e = 0; e < b->nenv; e++) t += h[(size_t)e * DX_NSTAGE + k];
    out[k] = t;
  }
  HIPCHK(hipStreamSynchronize(b->stream));
  return 0;
}
