// bf_check — TEST INFRASTRUCTURE.  Checks, on the CPU, the candidate closest-hit rule of the
// whole-wave trace (ray-tracing-c_amd/csrc/rt_book1.h: bf_trace) against the reference's traversal
// order (src/hittable.c:74-88 HittableList_hit, :266-277 BVHNode_hit, :38-55 AABB_hit, :120-151
// Sphere_hit) over the same preorder items the kernel uses, for a large set of rays of a reference
// scene: camera rays (with the scene's defocus disc) and rays leaving their hit points in random
// and mirror directions, as the paths do.  IEEE single precision without contraction, as on the GPU
// (whose fast sqrt/div cores are bitwise equal to these operators, tests/test_libm_port.py).
// Prints "rays decided undecided mismatches"; a mismatch (decided but different from the scan) is
// a bug.  Not part of the product.
//   bf_check <scene> <width> <n_rays> <seed>
#include "../../include/rt_hip.h"

#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <functional>
#include <vector>

struct Item {
  float q0[4], q1[4];
  bool leaf;
  uint32_t skip;  // node: 1 + subtree items
  int sphere;
};

static long dq_ref_steps, dq_steps, dq_rollbacks;  // (the deferred trace's counters, below)

struct Ray {
  float o[3], d[3], inv[3], a;
};

static void build(const rt_flat_scene *s, std::vector<Item> &items) {
  const rt_list &root = s->lists[rt_ref_index(s->root)];
  std::function<void(int32_t)> emit = [&](int32_t ref) {
    if (ref == RT_REF_NONE) return;
    const int32_t i = rt_ref_index(ref);
    Item it = {};
    if (rt_ref_kind(ref) == RT_KIND_SPHERE) {
      const rt_sphere &sp = s->spheres[i];
      it.q0[0] = sp.center[0], it.q0[1] = sp.center[1], it.q0[2] = sp.center[2], it.q0[3] = sp.radius_sq;
      it.leaf = true, it.sphere = i;
      items.push_back(it);
      return;
    }
    const rt_bvh_node &n = s->bvh[i];
    it.q0[0] = n.lo[0], it.q0[1] = n.hi[0], it.q0[2] = n.lo[1], it.q0[3] = n.hi[1];
    it.q1[0] = n.lo[2], it.q1[1] = n.hi[2];
    const size_t at = items.size();
    items.push_back(it);
    emit(n.left);
    emit(n.right);
    items[at].skip = (uint32_t)(items.size() - at);
  };
  for (int k = 0; k < root.count; k++) emit(s->list_items[root.first + k]);
}

// Sphere_hit's accepted root independent of t_max: q1, or q2 when q1 <= t_min; -inf: no root
static float sphere_root(const Item &it, const Ray &R, float tmin) {
  const float ocx = R.o[0] - it.q0[0], ocy = R.o[1] - it.q0[1], ocz = R.o[2] - it.q0[2];
  const float b = (ocx * R.d[0] + ocy * R.d[1]) + ocz * R.d[2];
  const float c = ((ocx * ocx + ocy * ocy) + ocz * ocz) - it.q0[3];
  const float disc = b * b - R.a * c;
  if (disc < 0) return -INFINITY;
  const float sq = sqrtf(disc);
  const float q1 = (-b - sq) / R.a, q2 = (-b + sq) / R.a;
  return q1 <= tmin ? q2 : q1;
}

static void box_interval(const Item &it, const Ray &R, float tmin, float *e, float *x) {
  const float t0x = (it.q0[0] - R.o[0]) * R.inv[0], t1x = (it.q0[1] - R.o[0]) * R.inv[0];
  const float t0y = (it.q0[2] - R.o[1]) * R.inv[1], t1y = (it.q0[3] - R.o[1]) * R.inv[1];
  const float t0z = (it.q1[0] - R.o[2]) * R.inv[2], t1z = (it.q1[1] - R.o[2]) * R.inv[2];
  const float nx = R.inv[0] < 0 ? t1x : t0x, fx = R.inv[0] < 0 ? t0x : t1x;
  const float ny = R.inv[1] < 0 ? t1y : t0y, fy = R.inv[1] < 0 ? t0y : t1y;
  const float nz = R.inv[2] < 0 ? t1z : t0z, fz = R.inv[2] < 0 ? t0z : t1z;
  *e = fmaxf(fmaxf(fmaxf(tmin, nx), ny), nz);
  *x = fminf(fminf(fx, fy), fz);
}

// the reference: AABB_hit slab by slab with early exit, then the sphere two-root sequence
static bool aabb_ref(const Item &it, const Ray &R, float tmin, float tmax) {
  const float lo[3] = {it.q0[0], it.q0[2], it.q1[0]}, hi[3] = {it.q0[1], it.q0[3], it.q1[1]};
  for (int i = 0; i < 3; i++) {
    const float inv = 1.0f / R.d[i];
    float t0 = (lo[i] - R.o[i]) * inv, t1 = (hi[i] - R.o[i]) * inv;
    if (inv < 0) {
      const float t = t0;
      t0 = t1, t1 = t;
    }
    tmin = fmaxf(tmin, t0);
    tmax = fminf(tmax, t1);
    if (tmax <= tmin) return false;
  }
  return true;
}
static bool sphere_ref(const Item &it, const Ray &R, float tmin, float tmax, float *t) {
  const float ocx = R.o[0] - it.q0[0], ocy = R.o[1] - it.q0[1], ocz = R.o[2] - it.q0[2];
  const float b = (ocx * R.d[0] + ocy * R.d[1]) + ocz * R.d[2];
  const float c = ((ocx * ocx + ocy * ocy) + ocz * ocz) - it.q0[3];
  const float disc = b * b - R.a * c;
  if (disc < 0) return false;
  const float sq = sqrtf(disc);
  float root = (-b - sq) / R.a;
  if (root <= tmin || root >= tmax) {
    root = (-b + sq) / R.a;
    if (root <= tmin || root >= tmax) return false;
  }
  *t = root;
  return true;
}
static void trace_ref(const std::vector<Item> &items, const Ray &R, float tmin, float *t, int *hit) {
  float tmax = INFINITY;
  *hit = -1;
  for (size_t p = 0; p < items.size(); dq_ref_steps++) {
    const Item &it = items[p];
    if (it.leaf) {
      float r;
      if (sphere_ref(it, R, tmin, tmax, &r)) tmax = r, *hit = it.sphere;
      p++;
    } else {
      p += aabb_ref(it, R, tmin, tmax) ? 1 : it.skip;
    }
  }
  *t = tmax;
}

// census: items the reference scan visits; nodes / leaves a t_max-free scan visits (every box with
// E < X entered); leaves under the depth-d boxes that pass t_max-free (the candidates of a cut filter)
static long cen_ref, cen_free_nodes, cen_free_leaves, cen_cut[10];
static bool pass_free(const Item &it, const Ray &R, float tmin) {
  float e, x;
  box_interval(it, R, tmin, &e, &x);
  return fminf(INFINITY, x) > e;
}
static void census(const std::vector<Item> &items, const Ray &R, float tmin) {
  float tmax = INFINITY;
  for (size_t p = 0; p < items.size();) {
    cen_ref++;
    const Item &it = items[p];
    if (it.leaf) {
      float r;
      if (sphere_ref(it, R, tmin, tmax, &r)) tmax = r;
      p++;
    } else {
      p += aabb_ref(it, R, tmin, tmax) ? 1 : it.skip;
    }
  }
  for (size_t p = 0; p < items.size();) {
    if (items[p].leaf) {
      cen_free_leaves++;
      p++;
    } else {
      cen_free_nodes++;
      p += pass_free(items[p], R, tmin) ? 1 : items[p].skip;
    }
  }
  for (int d = 1; d < 10; d++) {
    std::vector<size_t> ends;
    for (size_t p = 0; p < items.size();) {
      while (!ends.empty() && p >= ends.back()) ends.pop_back();
      const Item &it = items[p];
      if (it.leaf) {
        cen_cut[d]++;
        p++;
      } else if ((int)ends.size() == d) {  // a cut node: its leaves are candidates when it passes
        if (pass_free(it, R, tmin))
          for (size_t q = p; q < p + it.skip; q++) cen_cut[d] += items[q].leaf;
        p += it.skip;
      } else {
        ends.push_back(p + it.skip);
        p++;
      }
    }
  }
}

// bf_trace's rule; false = undecided (the kernel then runs the exact scan)
static bool trace_bf(const std::vector<Item> &items, const Ray &R, float tmin, float *t, int *hit) {
  float best = INFINITY;
  long bp = -1;
  for (size_t p = 0; p < items.size(); p++) {
    if (!items[p].leaf) continue;
    const float r = sphere_root(items[p], R, tmin);
    if (r != r) return false;
    if (r > tmin && r < best) best = r, bp = (long)p;
  }
  if (bp < 0) {
    *t = INFINITY, *hit = -1;
    return true;
  }
  for (long q = 0; q < bp; q++) {
    const Item &it = items[q];
    if (it.leaf || !(bp < q + (long)it.skip)) continue;
    float e, x;
    box_interval(it, R, tmin, &e, &x);
    if (!(fminf(best, x) > e)) return false;
  }
  *t = best, *hit = items[bp].sphere;
  return true;
}

// ---- the 8-wide form (group trace): a wide node holds the binary descendants 3 levels below a tested
// binary node (or the root list's items expanded 2 levels), each with its 0-2 intermediate nodes
struct WEntry {
  int item, child, n_inter, inter[3];
};
struct WNode {
  int n;
  WEntry e[8];
};
static std::vector<WNode> wide;
static int children(const std::vector<Item> &items, int p, int out[2]) {
  const int l = p + 1, ls = items[l].leaf ? 1 : (int)items[l].skip;
  int n = 0;
  out[n++] = l;
  if (l + ls < p + (int)items[p].skip) out[n++] = l + ls;
  return n;
}
static int g_max_inter = 3;
// greedy treelet: start from the level-1 items, then repeatedly open the internal entry with the
// largest subtree (it becomes an intermediate of its children) while the node has room
static int make_wide(const std::vector<Item> &items, const std::vector<int> &level1) {
  WNode w = {};
  if (level1.size() > 8) return -1;
  for (int c : level1) {
    WEntry &e = w.e[w.n++];
    e.item = c, e.child = -1, e.n_inter = 0, e.inter[0] = e.inter[1] = -1;
  }
  for (;;) {
    int pick = -1;
    for (int k = 0; k < w.n; k++) {
      const WEntry &e = w.e[k];
      if (items[e.item].leaf || e.n_inter >= g_max_inter) continue;
      int kc[2];
      if (w.n + children(items, e.item, kc) - 1 > 8) continue;
      if (pick < 0 || items[e.item].skip > items[w.e[pick].item].skip) pick = k;
    }
    if (pick < 0) break;
    const WEntry old = w.e[pick];
    int kc[2];
    const int nc = children(items, old.item, kc);
    for (int k = w.n - 1; k > pick; k--) w.e[k + nc - 1] = w.e[k];  // keep preorder
    for (int c = 0; c < nc; c++) {
      WEntry &e = w.e[pick + c];
      e = old;
      e.item = kc[c];
      e.inter[e.n_inter++] = old.item;
    }
    w.n += nc - 1;
  }
  const int id = (int)wide.size();
  wide.push_back(w);
  for (int k = 0; k < w.n; k++) {
    const int it = w.e[k].item;
    if (items[it].leaf) continue;
    int kc[2];
    const int nc = children(items, it, kc);
    const int c = make_wide(items, std::vector<int>(kc, kc + nc));
    if (c < 0) return -1;
    wide[id].e[k].child = c;
  }
  return id;
}
static long wide_iters;
static bool trace_wide(const std::vector<Item> &items, const Ray &R, float tmin, float *t, int *hit) {
  float best = INFINITY, best_e = -INFINITY;
  long bp = -1;
  std::vector<std::pair<int, float>> stack = {{0, -INFINITY}};
  while (!stack.empty()) {
    const auto [wi, me] = stack.back();
    stack.pop_back();
    wide_iters++;
    const WNode &w = wide[wi];
    for (int k = 0; k < w.n; k++) {
      const WEntry &e = w.e[k];
      float emax = me;
      bool ok = true;
      for (int q = 0; q < e.n_inter; q++) {
        float ee, xx;
        box_interval(items[e.inter[q]], R, tmin, &ee, &xx);
        ok &= fminf(INFINITY, xx) > ee;
        emax = fmaxf(emax, ee);
      }
      if (!ok) continue;
      if (items[e.item].leaf) {
        const float r = sphere_root(items[e.item], R, tmin);
        if (r != r) return false;
        if (r > tmin && (r < best || (r == best && e.item < bp))) best = r, bp = e.item, best_e = emax;
      } else {
        float ee, xx;
        box_interval(items[e.item], R, tmin, &ee, &xx);
        if (fminf(INFINITY, xx) > ee) stack.push_back({e.child, fmaxf(emax, ee)});
      }
    }
  }
  if (bp < 0) {
    *t = INFINITY, *hit = -1;
    return true;
  }
  if (!(best_e < best)) return false;
  *t = best, *hit = items[bp].sphere;
  return true;
}

static uint64_t rng_state;
static float frand() {  // [0,1)
  rng_state = rng_state * 6364136223846793005ULL + 1442695040888963407ULL;
  return (float)(rng_state >> 40) * 0x1p-24f;
}

static void set_ray(Ray &R, const float o[3], const float d[3]) {
  for (int i = 0; i < 3; i++) R.o[i] = o[i], R.d[i] = d[i], R.inv[i] = 1.0f / d[i];
  R.a = (d[0] * d[0] + d[1] * d[1]) + d[2] * d[2];
}

// The deferred sphere tests tried in r06 (profiles/r06/leaf_defer_experiment.patch: trav_step_defer / defer_drain):
// a leaf waits in the lane's one slot while the walk goes on over boxes with the stale t_max, until a
// random delay of up to `window` steps runs out, the walk reaches the next leaf (that step is lost) or
// the end; a deferred hit sends the walk back to the leaf's successor.  Must give the reference's hit
// bit for bit under any drain schedule; counts the steps it takes against the reference scan's.
static void trace_defer(const std::vector<Item> &items, const Ray &R, float tmin, int window, float *t, int *hit) {
  float tmax = INFINITY;
  *hit = -1;
  long pend = -1;
  int wait = 0;
  size_t p = 0;
  for (;;) {
    bool drain = false;
    if (p >= items.size()) {
      if (pend < 0) break;
      drain = true;
    } else {
      dq_steps++;
      const Item &it = items[p];
      if (it.leaf) {
        if (pend >= 0) {
          drain = true;  // blocked: the slot is taken
        } else {
          pend = (long)p;
          wait = window > 0 ? (int)(frand() * (float)(window + 1)) : 0;
          p++;
        }
      } else {
        p += aabb_ref(it, R, tmin, tmax) ? 1 : it.skip;
      }
      if (pend >= 0 && wait-- <= 0) drain = true;
    }
    if (drain && pend >= 0) {
      float r;
      if (sphere_ref(items[pend], R, tmin, tmax, &r)) {
        tmax = r, *hit = items[pend].sphere;
        p = (size_t)pend + 1;
        dq_rollbacks++;
      }
      pend = -1;
    }
  }
  *t = tmax;
}

int main(int argc, char **argv) {
  if (argc < 5) {
    fprintf(stderr, "usage: bf_check <scene> <width> <n_rays> <seed>\n");
    return 2;
  }
  rt_flat_scene *s = rt_scene_preset(atoi(argv[1]), atoi(argv[2]), 1, 50);
  if (!s) return 1;
  const long n_rays = atol(argv[3]);
  rng_state = strtoull(argv[4], nullptr, 10) * 2 + 1;
  std::vector<Item> items;
  build(s, items);
  std::vector<int> tops;
  for (int p = 0; p < (int)items.size(); p += items[p].leaf ? 1 : (int)items[p].skip) tops.push_back(p);
  const bool wide_ok = make_wide(items, tops) == 0;
  long w_dec = 0, w_und = 0, w_bad = 0;
  const rt_camera &c = s->camera;
  const float tmin = 1e-3f;
  long decided = 0, undecided = 0, bad = 0, hits = 0, d_bad = 0;
  for (long k = 0; k < n_rays;) {
    // a camera ray through a random pixel position, with the defocus disc
    const float fi = frand() * (float)c.width, fj = frand() * (float)c.height;
    float o[3], d[3];
    const float a = 2.0f * frand() - 1.0f, b = 2.0f * frand() - 1.0f;
    for (int i = 0; i < 3; i++) {
      o[i] = c.origin[i] + (c.dof_angle > 0.0f ? c.disc_u[i] * a + c.disc_v[i] * b : 0.0f);
      d[i] = (c.pixel00[i] + c.delta_u[i] * fi + c.delta_v[i] * fj) - o[i];
    }
    for (int bounce = 0; bounce < 6 && k < n_rays; bounce++) {
      k++;
      Ray R;
      set_ray(R, o, d);
      float t_ref, t_bf;
      int h_ref, h_bf;
      trace_ref(items, R, tmin, &t_ref, &h_ref);
      if (getenv("BF_CENSUS")) census(items, R, tmin);
      if (const char *dw = getenv("BF_DEFER")) {
        float t_d;
        int h_d;
        trace_defer(items, R, tmin, atoi(dw), &t_d, &h_d);
        if (h_d != h_ref || (h_ref >= 0 && t_d != t_ref)) {
          if (d_bad < 10) fprintf(stderr, "deferred mismatch: ref %d %a, deferred %d %a\n", h_ref, t_ref, h_d, t_d);
          d_bad++;
        }
      }
      if (trace_bf(items, R, tmin, &t_bf, &h_bf)) {
        decided++;
        if (h_bf != h_ref || (h_ref >= 0 && t_bf != t_ref)) {
          if (bad < 10)
            fprintf(stderr, "mismatch: ray o=(%a %a %a) d=(%a %a %a): ref %d %a, bf %d %a\n", o[0], o[1], o[2], d[0],
                    d[1], d[2], h_ref, t_ref, h_bf, t_bf);
          bad++;
        }
      } else {
        undecided++;
      }
      if (wide_ok) {
        if (trace_wide(items, R, tmin, &t_bf, &h_bf)) {
          w_dec++;
          if (h_bf != h_ref || (h_ref >= 0 && t_bf != t_ref)) w_bad++;
        } else {
          w_und++;
        }
      }
      if (h_ref < 0) break;
      hits++;
      // continue from the hit point: a random direction (half of the time) or a mirror one
      const rt_sphere &sp = s->spheres[h_ref];
      float p[3], n[3], dn = 0.0f;
      for (int i = 0; i < 3; i++) p[i] = o[i] + d[i] * t_ref, n[i] = (p[i] - sp.center[i]) / sp.radius;
      for (int i = 0; i < 3; i++) dn += d[i] * n[i];
      if (frand() < 0.5f) {
        for (int i = 0; i < 3; i++) d[i] = d[i] - 2.0f * dn * n[i] + 0.3f * (2.0f * frand() - 1.0f);
      } else {
        float u[3], l2;
        do {
          for (int i = 0; i < 3; i++) u[i] = 2.0f * frand() - 1.0f;
          l2 = u[0] * u[0] + u[1] * u[1] + u[2] * u[2];
        } while (l2 >= 1.0f || l2 == 0.0f);
        const float sgn = dn < 0 ? 1.0f : -1.0f;  // scatter to the incoming side
        for (int i = 0; i < 3; i++) d[i] = sgn * n[i] + u[i] / sqrtf(l2);
      }
      for (int i = 0; i < 3; i++) o[i] = p[i];
    }
  }
  printf("%ld %ld %ld %ld\n", n_rays, decided, undecided, bad);
  fprintf(stderr, "rays %ld: decided %ld, undecided %ld (%.4f%%), mismatches %ld, hit rays %ld\n", n_rays, decided,
          undecided, 100.0 * undecided / (double)n_rays, bad, hits);
  fprintf(stderr, "wide (8-wide group trace): %s, %zu nodes; decided %ld, undecided %ld, mismatches %ld, %.2f nodes/ray\n",
          wide_ok ? "built" : "not buildable", wide.size(), w_dec, w_und, w_bad, (double)wide_iters / n_rays);
  bad += w_bad;
  if (getenv("BF_DEFER")) {
    fprintf(stderr, "deferred sphere tests (window %s): mismatches %ld; steps %.2f per ray against the reference scan's %.2f "
            "(x%.3f), rollbacks %.3f per ray\n", getenv("BF_DEFER"), d_bad, (double)dq_steps / n_rays,
            (double)dq_ref_steps / n_rays, (double)dq_steps / (double)dq_ref_steps, (double)dq_rollbacks / n_rays);
    bad += d_bad;
  }
  if (getenv("BF_CENSUS")) {
    fprintf(stderr, "per ray: reference scan %.1f items; t_max-free scan %.1f nodes, %.1f leaves; cut candidates",
            (double)cen_ref / n_rays, (double)cen_free_nodes / n_rays, (double)cen_free_leaves / n_rays);
    for (int d = 1; d < 10; d++) fprintf(stderr, " d%d:%.1f", d, (double)cen_cut[d] / n_rays);
    fprintf(stderr, "\n");
  }
  rt_flat_free(s);
  return bad != 0;
}
