// volumetric.h — VolumetricDisc on gfx950 (src/scene_objects/volumetric_disc.rs).
// Included once by geodesic.hip, after the shading helpers it uses.
//
// Window test (integrate_kernel): the capture region is the annulus rin..rout of
// half-height 3*thickness around the axis; Hittable::intersects (:506-578) returns the
// first crossing of its boundary (two clipped cylinders + two caps, :348-494) with
// t > 1e-9.  The candidate keeps the world hit point and the chord direction.
//
// Colour (march_kernel): VolumetricDisc::color_at_uv raymarches from the hit point
// along the normalised chord (:580-601, :199-328) with a constant step: per sample
// the Perlin-fBm density (:97-138), Beer-Lambert attenuation, and -- where a timelike
// circular orbit exists -- the per-sample redshift from the conserved (p_t, p_phi),
// the disc temperature, the texture colour and T^4 emission.  Up to max_steps (50000
// in the stock scenes) samples per hit, so it runs as its own persistent kernel over a
// compacted job list, with the same lane-refill scheme as integrate_kernel.
//
// Arithmetic follows the reference's evaluation order (nalgebra Vector3: dot = a + b
// + c, cross, norm = sqrt(dot), v / s per component); exp() and pow() return glibc's
// bits (glibc_math.h), sin/cos of one angle are glibc's sincos; atan2 is the device's.
// Perlin noise is noise 0.9.0's perlin_3d with the host-built permutation table
// (host/volumetric.cpp), staged in LDS.
// (Included inside namespace grt.)
#pragma once

struct V3 {
  double x, y, z;
};
GDEV double vdot(const V3& a, const V3& b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
GDEV V3 vcross(const V3& a, const V3& b) {
  return V3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
GDEV V3 vsub(const V3& a, const V3& b) { return V3{a.x - b.x, a.y - b.y, a.z - b.z}; }
GDEV V3 vmad(const V3& a, double t, const V3& d) { return V3{a.x + t * d.x, a.y + t * d.y, a.z + t * d.z}; }
GDEV V3 vaxis(const DevObject& o) { return V3{o.ax[0], o.ax[1], o.ax[2]}; }
GDEV double vnorm(const V3& a) { return sqrt(vdot(a, a)); }

// f64::total_cmp order key
GDEV uint64_t total_key(double x) {
  const uint64_t u = glibc::as_u64(x);
  return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}

// ---- capture-region boundary (volumetric_disc.rs:348-494) -------------------------
// intersects_clipped_cylinder: crossings of |x × axis| = radius with |x·axis| <= hh,
// as segment fractions t (0, 1 or 2 of them, ascending).
GDEV int clipped_cylinder(const DevObject& o, const V3& from, const V3& to, double radius, double hh,
                          double* t_out) {
  const V3 sv = vsub(to, from);
  const double len = vnorm(sv);
  if (len < 1e-12) return 0;
  const V3 d{sv.x / len, sv.y / len, sv.z / len};
  const V3 ax = vaxis(o);
  const V3 v = vcross(from, ax);
  const V3 w = vcross(d, ax);
  const double a = vdot(w, w);
  const double b = 2.0 * vdot(v, w);
  const double c = vdot(v, v) - radius * radius;
  if (a < 1e-10) return 0;  // Parallel / NoIntersection: both ignored by the caller
  const double disc = b * b - 4.0 * a * c;
  if (disc < 0.0) return 0;
  const double sq = sqrt(disc);
  const double dists[2] = {(-b - sq) / (2.0 * a), (-b + sq) / (2.0 * a)};
  int n = 0;
  double h[2] = {0.0, 0.0};
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const double t = dists[k] / len;
    if (0.0 <= t && t <= 1.0) {
      const V3 p = vmad(from, t, sv);
      if (fabs(vdot(p, ax)) <= hh) h[n++] = t;
    }
  }
  if (n == 2) {
    t_out[0] = fmin(h[0], h[1]);
    t_out[1] = fmax(h[0], h[1]);
  } else if (n == 1) {
    t_out[0] = h[0];
  }
  return n;
}

// intersects_cap: the plane x·axis = pos inside radius
GDEV bool cap_hit(const DevObject& o, const V3& from, const V3& to, double radius, double pos, double* t_out) {
  const V3 sv = vsub(to, from);
  const double len = vnorm(sv);
  if (len < 1e-12) return false;
  const V3 ax = vaxis(o);
  const V3 n{sv.x / len, sv.y / len, sv.z / len};
  if (fabs(vdot(n, ax)) < 1e-10) return false;
  const double t = (pos - vdot(from, ax)) / vdot(sv, ax);
  if (!(0.0 <= t && t <= 1.0)) return false;
  const V3 p = vmad(from, t, sv);
  const V3 c = vcross(p, ax);
  if (vdot(c, c) > radius * radius) return false;
  *t_out = t;
  return true;
}

// intersects_cylinder: all boundary crossings, sorted by total_cmp; returns how many
// (0, 1, or 2 = at least two, the two smallest in t[0] <= t[1]).
GDEV int capture_crossings(const DevObject& o, const V3& from, const V3& to, double* t) {
  double hits[6];
  int n = 0;
  double c2[2];
  int k = clipped_cylinder(o, from, to, o.rout, o.cap_h, c2);
  for (int i = 0; i < k; ++i) hits[n++] = c2[i];
  k = clipped_cylinder(o, from, to, o.rin, o.cap_h, c2);
  for (int i = 0; i < k; ++i) hits[n++] = c2[i];
  const V3 dir = vsub(to, from);
  const V3 ax = vaxis(o);
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const double pos = s == 0 ? o.cap_h : -o.cap_h;
    double tc;
    if (cap_hit(o, from, to, o.rout, pos, &tc)) {
      const V3 p = vmad(from, tc, dir);
      const V3 c = vcross(p, ax);
      if (vdot(c, c) >= o.rin2) hits[n++] = tc;
    }
  }
  if (n == 0) return 0;
  int i0 = 0;  // the two smallest under total_cmp
  for (int i = 1; i < n; ++i)
    if (total_key(hits[i]) < total_key(hits[i0])) i0 = i;
  t[0] = hits[i0];
  if (n == 1) return 1;
  int i1 = i0 == 0 ? 1 : 0;
  for (int i = 0; i < n; ++i)
    if (i != i0 && total_key(hits[i]) < total_key(hits[i1])) i1 = i;
  t[1] = hits[i1];
  return 2;
}

// Hittable::intersects (:506-578): the first crossing with t > 1e-9 (t in [0, 1]).
GDEV bool vdisc_chord(const DevObject& o, const double* s, const double* e, double* t_out, double* ip) {
  const V3 from{s[0], s[1], s[2]}, to{e[0], e[1], e[2]};
  double t2[2];
  const int n = capture_crossings(o, from, to, t2);
  double t;
  if (n == 0) return false;
  if (n == 1) {
    if (!(t2[0] > 1e-9)) return false;
    t = t2[0];
  } else if (t2[0] > 1e-9) {
    t = t2[0];
  } else if (t2[1] > 1e-9) {
    t = t2[1];
  } else {
    return false;
  }
  if (!(0.0 <= t && t <= 1.0)) return false;
  const V3 p = vmad(from, t, vsub(to, from));
  *t_out = t;
  ip[0] = p.x;
  ip[1] = p.y;
  ip[2] = p.z;
  return true;
}

// ---- Perlin noise (noise 0.9.0 core/perlin.rs perlin_3d) -------------------------
// hash: P[P[P[x & 255] ^ (y & 255)] ^ (z & 255)]; gradient_dot_v picks +-u +-v:
//   h   0..7: u = x        8..11: u = y      12,13: u = x      14,15: u = y
//   v   0..3: y   4..11: z   12,13: y   14,15: z;   -u: h odd or h >= 14;
//   -v: (h & 2) for h < 12, and h == 15.   (-x) + y etc. are exact negations.
GDEV double s_curve5(double x) { return x * x * x * (x * (x * 6.0 - 15.0) + 10.0); }

// grad_dot as coefficients: hash h picks (gx, gy, gz) in {-1, 0, +1}, two of them non-zero
// (+-u +- v above), and gradient_dot_v is fma(gz, z, fma(gy, y, gx * x)).  Each product
// is exact (x, -x or a zero), so the two fused adds round the exact sum +-u +- v once, as
// the reference's one addition does: the same value, except that a zero result may carry
// the other sign.  That never reaches the density: every perlin value only enters the
// fBm sum n, which starts at +0.0 and is never -0.0, and x + (+-0) is x for every x != 0
// and +0 for x = +0.  The march kernel keeps the 16 rows in LDS (one read of a 32-B row
// per corner instead of ~26 integer / select instructions of grad_dot).
GDEV double grad_coef(uint32_t h, uint32_t axis) {
  h &= 15u;
  const uint32_t u_axis = (h < 8u || h == 12u || h == 13u) ? 0u : 1u;
  const uint32_t v_axis = (h < 4u || h == 12u || h == 13u) ? 1u : 2u;
  const bool nu = (h & 1u) || h >= 14u;
  const bool nv = h < 12u ? (h & 2u) != 0u : h == 15u;
  if (axis == u_axis) return nu ? -1.0 : 1.0;
  if (axis == v_axis) return nv ? -1.0 : 1.0;
  return 0.0;
}
GDEV double grad_dot_lds(const double* __restrict__ G, uint32_t h, double x, double y, double z) {
  const double* g = G + ((h & 15u) << 2);
  return __builtin_fma(g[2], z, __builtin_fma(g[1], y, g[0] * x));
}

// (corner as isize) & 0xff of an integral double: fl - 256 floor(fl / 256) is exact
// (power-of-two scaling, integral operands below 2^53) and lies in [0, 255]; the
// reference's numcast() panics beyond the isize range, where this is never reached.
GDEV uint32_t lattice_byte(double fl) { return (uint32_t)(int32_t)__builtin_fma(-256.0, floor(fl * 0.00390625), fl); }

GDEV double perlin3(const uint8_t* P, const double* G, double px, double py, double pz) {
  const double fx = floor(px), fy = floor(py), fz = floor(pz);
  const double dx = px - fx, dy = py - fy, dz = pz - fz;
  const uint32_t x0 = lattice_byte(fx), x1 = (x0 + 1u) & 0xffu;
  const uint32_t y0 = lattice_byte(fy), y1 = (y0 + 1u) & 0xffu;
  const uint32_t z0 = lattice_byte(fz), z1 = (z0 + 1u) & 0xffu;
  const uint32_t a0 = P[x0], a1 = P[x1];
  const uint32_t b00 = P[a0 ^ y0], b10 = P[a1 ^ y0], b01 = P[a0 ^ y1], b11 = P[a1 ^ y1];
  const double dx1 = dx - 1.0, dy1 = dy - 1.0, dz1 = dz - 1.0;
  const double g000 = grad_dot_lds(G, P[b00 ^ z0], dx, dy, dz);
  const double g100 = grad_dot_lds(G, P[b10 ^ z0], dx1, dy, dz);
  const double g010 = grad_dot_lds(G, P[b01 ^ z0], dx, dy1, dz);
  const double g110 = grad_dot_lds(G, P[b11 ^ z0], dx1, dy1, dz);
  const double g001 = grad_dot_lds(G, P[b00 ^ z1], dx, dy, dz1);
  const double g101 = grad_dot_lds(G, P[b10 ^ z1], dx1, dy, dz1);
  const double g011 = grad_dot_lds(G, P[b01 ^ z1], dx, dy1, dz1);
  const double g111 = grad_dot_lds(G, P[b11 ^ z1], dx1, dy1, dz1);
  const double a = s_curve5(dx), b = s_curve5(dy), c = s_curve5(dz);
  const double k0 = g000;
  const double k1 = g100 - g000;
  const double k2 = g010 - g000;
  const double k3 = g001 - g000;
  const double k4 = g000 + g110 - g100 - g010;
  const double k5 = g000 + g101 - g100 - g001;
  const double k6 = g000 + g011 - g010 - g001;
  const double k7 = g100 + g010 + g001 + g111 - g000 - g110 - g101 - g011;
  const double r = k0 + k1 * a + k2 * b + k3 * c + k4 * a * b + k5 * a * c + k6 * b * c + k7 * a * b * c;
  return rclamp(r * 1.1547005383792515, -1.0, 1.0);
}

// ---- density, uv (volumetric_disc.rs:97-152) -------------------------------------
// Also returns the in-plane coordinates (x_local, y_local) and sin / cos of their angle
// phi when the noise was evaluated (*noise): get_uv (:140-152) recomputes exactly these
// values at the same point, so the raymarch reuses them.
struct PlaneAngle {
  double x, y, sp, cp;
};
GDEV double vdisc_density(const DevObject& o, const uint8_t* P, const double* G, const V3& p, PlaneAngle* pa,
                          bool* noise) {
  *noise = false;
  const V3 ax = vaxis(o);
  const double h = fabs(vdot(p, ax));
  const double r = vnorm(vcross(p, ax));
  if (r <= o.rin || r >= o.rout) return 0.0;
  const double q = h / o.thickness;
  const double vertical_falloff = glibc::exp_(-(q * q));
  if (vertical_falloff < 0.001) return 0.0;
  const double radial_base = rpow(o.rin / r, 1.5);
  double boundary_falloff = 1.0;
  const double d1 = o.rout - r, d2 = r - o.rin;
  boundary_falloff *= glibc::exp_(-1.0 / fmax(d1 * d1, 0.0001));
  boundary_falloff *= glibc::exp_(-1.0 / fmax(d2 * d2, 0.0001));
  const V3 e1{o.e1[0], o.e1[1], o.e1[2]}, e2{o.e2[0], o.e2[1], o.e2[2]};
  const double x_local = vdot(p, e1), y_local = vdot(p, e2);
  const double phi = atan2(y_local, x_local);
  double sp, cp;  // phi is spread over (-pi, pi] within a wave: the branch-free sincos
  if (!glibc::sincos_fast_uniform(phi, &sp, &cp)) sincos(phi, &sp, &cp);
  *noise = true;
  *pa = PlaneAngle{x_local, y_local, sp, cp};
  const double npx = r * o.ns[0], npy = cp * o.ns[1], npz = sp * o.ns[1];
  double n = 0.0, frequency = 4.0, amplitude = 1.0;  // fbm (:330-342)
  for (uint32_t i = 0; i < o.octaves; ++i) {
    n += amplitude * perlin3(P, G, npx * frequency, npy * frequency, npz * frequency);
    frequency *= 2.0;
    amplitude *= o.g_fbm;
  }
  n += perlin3(P, G, r * 0.5, h * o.ns[2], cp) * 0.5;
  const double n2 = fmax(n + o.noff, 0.0) * o.dens_mult;
  return n2 * radial_base * vertical_falloff * boundary_falloff;
}

// get_uv from the density's PlaneAngle (same point: the same x, y, phi, sin, cos)
GDEV void vdisc_uv(const DevObject& o, const PlaneAngle& pa, double* u, double* v) {
  const double rr = sqrt(pa.x * pa.x + pa.y * pa.y);
  const double r = (rr - o.rin) / (o.rout - o.rin);
  *u = 0.5 + 0.5 * r * pa.cp;
  *v = 0.5 + 0.5 * r * pa.sp;
}

// precompute_exit_distance (:172-196): distance to the first boundary crossing (t > 1e-9)
// within max_steps * step_size; false = none (the march then tests does_exit per sample).
GDEV bool vdisc_exit_distance(const DevObject& o, const V3& ro, const V3& rd, double* out) {
  const double md = o.m_maxdist;
  const V3 to{ro.x + rd.x * md, ro.y + rd.y * md, ro.z + rd.z * md};
  double t[2];
  const int n = capture_crossings(o, ro, to, t);
  if (n >= 1 && t[0] > 1e-9) {
    *out = t[0] * md;
    return true;
  }
  if (n >= 2 && t[1] > 1e-9) {
    *out = t[1] * md;
    return true;
  }
  return false;
}

// Geometry::circular_orbit_killing_coefficients of a Cartesian sample (euclidean.rs:207-217,
// schwarzschild.rs:260-265 with |p|, kerr.rs:487-496 / kerr_bl.rs:398-410 with the BL r)
template <int G>
GDEV bool killing_at(const DevScene& S, const V3& p, double* ut, double* uphi) {
  if constexpr (G == GRT_GEOM_EUCLIDEAN || G == GRT_GEOM_EUCLIDEAN_SPHERICAL) {
    *ut = 1.0;
    *uphi = 0.0;
    return true;
  } else {
    double r;
    if constexpr (G == GRT_GEOM_SCHWARZSCHILD) r = sqrt(p.x * p.x + p.y * p.y + p.z * p.z);
    else r = sqrt(ks_r_sqr(S.a, p.x, p.y, p.z));
    return killing_coefficients(S, r, ut, uphi);
  }
}

// True when no sample at or beyond p (along rd) can have density > 0, so the rest of
// the raymarch adds nothing: the colour is final whatever the exit test or max_steps
// would decide later.  Density needs rin < |p x axis| < rout and a vertical falloff
// exp(-(h/thickness)^2) >= 0.001, i.e. |h| <= 2.62826 thickness (vol_h_cut carries a
// 1e-6 margin).  h is linear along the ray and |p x axis|^2 convex, so a sample beyond
// the cut that moves away from the mid-plane, or beyond rout that moves outward, stays
// outside.  The margins (1e-9 relative, 1e-9 absolute) exceed the rounding of the
// positions any later sample could compute (|p| <= |ro| + max_steps * step_size) by
// orders of magnitude; slopes within -1e-15 of zero count as non-approaching, which
// moves h or r^2 by < 1e-12 over the whole march.
//   Most raymarch jobs start where a window LEAVES the capture region (volumetric_
// disc.rs:540-548 returns that crossing too): they march outward through empty space
// for up to max_steps samples, and end on the first sample here.
GDEV bool vdisc_no_more_density(const DevObject& o, const V3& p, const V3& rd) {
  const V3 ax = vaxis(o);
  const double pn = fabs(p.x) + fabs(p.y) + fabs(p.z);
  const double tol = 1e-9 * (1.0 + pn + o.m_maxdist);
  const double h = vdot(p, ax), s = vdot(rd, ax);
  if (fabs(h) > o.vol_h_cut + tol && (h > 0.0 ? s : -s) >= -1e-15) return true;
  const V3 c = vcross(p, ax), cd = vcross(rd, ax);
  const double r2 = vdot(c, c);
  const double rmin = o.rout + tol;
  return r2 > rmin * rmin && vdot(c, cd) >= -1e-15 * (1.0 + pn);
}

// ---- march kernel: one lane per job, refilled by wave ballot -----------------------
// Job = (ray slot << 8) | candidate slot, colour to ws.vcol at the candidate slot; or
// JOB_POOL | ray << 31 | pool record, colour to the record's vcol.
// The per-sample table lookups (temperature LUT of the first volumetric object with one,
// the blackbody LUT; lut_index) are staged in LDS (48 KB).
constexpr uint32_t MARCH_LUT_MAX = 1000;
template <int G>
__global__ void __launch_bounds__(256, 2) march_kernel(const DevScene* __restrict__ Sp, Workspace ws) {
  const DevScene& S = *Sp;
  __shared__ uint8_t lds_perm[GRT_MAX_OBJECTS * 256];
  __shared__ double lds_grad[16 * 4];  // grad_coef rows (gx, gy, gz, 0), 32 B each
  if (threadIdx.x < 64) lds_grad[threadIdx.x] = (threadIdx.x & 3u) == 3u ? 0.0 : grad_coef(threadIdx.x >> 2, threadIdx.x & 3u);
  __shared__ double lds_tr[MARCH_LUT_MAX], lds_tt[MARCH_LUT_MAX];
  __shared__ double lds_bt[MARCH_LUT_MAX], lds_bx[3 * MARCH_LUT_MAX];
  for (unsigned i = threadIdx.x; i < GRT_MAX_OBJECTS * 256u; i += blockDim.x) lds_perm[i] = S.perm[i >> 8][i & 255u];
  int lut_obj = -1;  // wave-uniform
  for (uint32_t q = 0; q < S.n_objects; ++q)
    if (lut_obj < 0 && S.obj[q].kind == GRT_OBJ_VOLUMETRIC_DISC && S.obj[q].temp_kind == GRT_TEMP_KERR_LUT &&
        S.obj[q].lut_n <= MARCH_LUT_MAX)
      lut_obj = (int)q;
  if (lut_obj >= 0) {
    const DevObject& lo = S.obj[lut_obj];
    for (unsigned i = threadIdx.x; i < lo.lut_n; i += blockDim.x) {
      lds_tr[i] = lo.lut_r[i];
      lds_tt[i] = lo.lut_t[i];
    }
  }
  const bool bb_lds = S.bb_n >= 2 && S.bb_n <= MARCH_LUT_MAX;
  if (bb_lds) {
    for (unsigned i = threadIdx.x; i < S.bb_n; i += blockDim.x) lds_bt[i] = S.bb_log_t[i];
    for (unsigned i = threadIdx.x; i < 3u * S.bb_n; i += blockDim.x) lds_bx[i] = S.bb_xyz[i];
  }
  const double* bb_lt = bb_lds ? lds_bt : S.bb_log_t;
  const double* bb_xyz = bb_lds ? lds_bx : S.bb_xyz;
  glibc::tables_to_lds();  // includes the block barrier
  const int lane = threadIdx.x & 63;
  const uint64_t lanemask_lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  const uint64_t n_jobs = ws.march[0];
  if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(ws.march + 3, (unsigned long long)n_jobs);
  const uint64_t n = ws.n;
  const uint64_t MN = (uint64_t)GRT_WS_SLOTS * n;
  constexpr uint64_t CHUNK = 64;
  uint64_t n_samples = 0, n_noise = 0, n_emit = 0;
  // One pass over the job list per VolumetricDisc of the scene, each with its own claim
  // cursor (ws.march[8 + kobj]): a pass marches only its object's jobs, so the object is
  // wave-uniform and its parameters sit in scalar registers (per-lane object loads held
  // ~80 VGPRs across the sample loop).  The stock scenes have one such object: one pass.
  for (uint32_t kobj = 0; kobj < S.n_objects; ++kobj) {
    if (S.obj[kobj].kind != GRT_OBJ_VOLUMETRIC_DISC) continue;
    const DevObject& o = S.obj[kobj];
    const uint8_t* P = lds_perm + o.perm_slot * 256u;
    const bool lds_t = (int)kobj == lut_obj;
    const double* lut_r = lds_t ? lds_tr : o.lut_r;
    const double* lut_t = lds_t ? lds_tt : o.lut_t;
    unsigned long long* cursor = ws.march + 8 + kobj;
    uint64_t chunk_next = 0, chunk_end = 0;
    bool active = false, done = false;
    // lane state
    uint64_t slot = 0, i = 0;
    V3 ro{0, 0, 0}, rd{0, 0, 0};
    double d_o = 0.0, exit_d = 0.0, transparency = 1.0, aws = 0.0, awt = 0.0;
    double acc_x = 0.0, acc_y = 0.0, acc_z = 0.0, obs = 0.0, f_pt = 0.0, f_pphi = 0.0;
    bool cached = false, pool_job = false;

    while (true) {
      bool need = !active && !done;
      uint64_t need_mask = __ballot(need);
      if (need_mask) {
        uint64_t cnt = __popcll(need_mask);
        uint64_t remaining = chunk_end - chunk_next;
        uint64_t new_base = 0;
        if (cnt > remaining) {
          unsigned long long b = 0;
          if (lane == 0) b = atomicAdd(cursor, (unsigned long long)CHUNK);
          new_base = __shfl(b, 0);
        }
        if (need) {
          uint64_t rank = __popcll(need_mask & lanemask_lt);
          uint64_t item = rank < remaining ? chunk_next + rank : new_base + (rank - remaining);
          if (item >= n_jobs) {
            done = true;
          } else {
            const uint64_t job = ws.jobs[item];
            pool_job = (job & JOB_POOL) != 0;
            uint64_t idx;
            uint32_t k;
            if (!pool_job) {
              idx = job >> 8;
              slot = (uint64_t)(uint32_t)(job & 255u) * n + idx;
              k = ws.rec[slot].obj;
            } else {  // a candidate past the workspace slots (HitPool record)
              idx = (job & ~JOB_POOL) >> 31;
              slot = job & 0x7fffffffull;
              k = ws.pool->obj[slot];
            }
            if (k == kobj) {  // another object's job waits for that object's pass
              V3 dir;
              if (!pool_job) {
                ro = V3{ws.rec[slot].pt[0], ws.rec[slot].pt[1], ws.rec[slot].pt[2]};
                dir = V3{ws.rec_dir[slot], ws.rec_dir[MN + slot], ws.rec_dir[2 * MN + slot]};
              } else {
                const uint64_t m = ws.pool->cap;
                ro = V3{ws.pool->pt[slot], ws.pool->pt[m + slot], ws.pool->pt[2 * m + slot]};
                dir = V3{ws.pool->dir[slot], ws.pool->dir[m + slot], ws.pool->dir[2 * m + slot]};
              }
              const double dn = vnorm(dir);  // .normalize()
              rd = V3{dir.x / dn, dir.y / dn, dir.z / dn};
              obs = ws.rc[idx];
              f_pt = ws.rc[4 * n + idx];
              f_pphi = ws.rc[5 * n + idx];
              cached = vdisc_exit_distance(o, ro, rd, &exit_d);
              d_o = 0.0;
              i = 0;
              transparency = 1.0;
              aws = awt = 0.0;
              acc_x = acc_y = acc_z = 0.0;
              active = true;
            }
          }
        }
        if (cnt > remaining) {
          chunk_next = new_base + (cnt - remaining);
          chunk_end = new_base + CHUNK;
        } else {
          chunk_next += cnt;
        }
      }
      if (__ballot(!done) == 0) break;
      if (!active) continue;

      // ---- one sample (raymarch_constant_step_internal, :234-309) ----
      const double d_s = o.m_step;
      const V3 p{ro.x + rd.x * d_o, ro.y + rd.y * d_o, ro.z + rd.z * d_o};
      d_o += d_s;
      n_samples++;
      bool failed = false;
      PlaneAngle pa;
      bool noise;
      const double density = vdisc_density(o, P, lds_grad, p, &pa, &noise);
      n_noise += noise ? 1u : 0u;
      if (density > 0.0) {
        const double sig = o.sig_a + o.sig_s;
        transparency *= glibc::exp_(-d_s * density * sig);
        double ut, uphi;
        if (killing_at<G>(S, p, &ut, &uphi)) {
          const double emitter_energy = ut * f_pt + uphi * f_pphi;
          const double redshift = obs / emitter_energy;
          const double r_dist = vnorm(vcross(p, vaxis(o)));
          double temperature;
          if (compute_temperature_lut(o, lut_r, lut_t, r_dist, &temperature) != GRT_OK) {
            failed = true;  // Err -> color_at_uv's unwrap_or_else: (0, 0, 0, 0)
          } else {
            n_emit++;
            double u, v;
            vdisc_uv(o, pa, &u, &v);
            const XYZA light = texture_color_lut(S, o.tex, u, v, redshift, temperature, bb_lt, bb_xyz);
            const double light_attenuation = glibc::exp_(-density * d_s * sig);
            const double ratio = temperature / o.bref;
            const double r2 = ratio * ratio;
            const double intensity = r2 * r2;  // powi(4)
            const double emission_weight = transparency * light_attenuation * o.sig_s * density * d_s;
            const double w = emission_weight * intensity;
            const double asw = density * d_s;
            aws += rclamp(light.a, 0.0, 1.0) * asw;
            awt += asw;
            acc_x += light.x * w;
            acc_y += light.y * w;
            acc_z += light.z * w;
          }
        }
      }
      bool finished = failed || (density == 0.0 && vdisc_no_more_density(o, p, rd));
      if (!finished) {
        bool exited;
        if (cached) {
          exited = d_o >= exit_d;
        } else {  // does_exit (:154-170): a crossing within this step
          const double st[3] = {p.x, p.y, p.z};
          const double end[3] = {p.x + rd.x * d_s, p.y + rd.y * d_s, p.z + rd.z * d_s};
          double tx, ipx[3];
          exited = vdisc_chord(o, st, end, &tx, ipx) && tx > 1e-9;
        }
        finished = exited || ++i >= o.m_max;
      }
      if (finished) {
        double col[4] = {0.0, 0.0, 0.0, 0.0};
        if (!failed) {
          const double physical_opacity = 1.0 - transparency;
          const double texture_alpha = awt > 0.0 ? aws / awt : 1.0;
          col[0] = acc_x;
          col[1] = acc_y;
          col[2] = acc_z;
          col[3] = physical_opacity * texture_alpha;
        }
        double* vc = pool_job ? ws.pool->vcol : ws.vcol;
        const uint64_t m = pool_job ? ws.pool->cap : MN;
#pragma unroll
        for (int q = 0; q < 4; ++q) vc[q * m + slot] = col[q];
        active = false;
      }
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    n_samples += __shfl_down(n_samples, off);
    n_noise += __shfl_down(n_noise, off);
    n_emit += __shfl_down(n_emit, off);
  }
  if (lane == 0) {
    atomicAdd(ws.march + 2, (unsigned long long)n_samples);
    atomicAdd(ws.march + 4, (unsigned long long)n_noise);
    atomicAdd(ws.march + 5, (unsigned long long)n_emit);
  }
}
