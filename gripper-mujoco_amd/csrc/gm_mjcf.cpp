// gm_mjcf.cpp -- MJCF loader / writer for the gripper model.
//
// The reference loads its gripper + task MJCF with mj_loadXML (mjclass.cpp:377-409), finds
// joints / bodies / geoms by name (JointSettings, myfunctions.cpp:166-464, 719-787; the
// object handler's name lists, objecthandler.cpp:22-133) and reads the gripper numerics
// from <custom><numeric> fields (read_gripper_dimensions, myfunctions.cpp:836-953).  The
// `description` submodule that generates those files is absent, so this module
//   - writes the compiled model (gm_build_model) as MJCF with the reference's naming
//     conventions (gm_model_to_mjcf), and
//   - compiles the MJCF subset that model uses back into a gm_model (gm_model_from_mjcf):
//     <option>, <default><geom solref solimp>, <custom><numeric>, the <worldbody> tree of
//     body / joint (slide, hinge, free) / inertial / geom (plane, sphere, cylinder, box),
//     <contact><pair>, <equality><joint> motor locks and the "initial pose" <keyframe>.
// Body / joint / dof / geom ids follow MuJoCo's compiler: depth-first document order.
// Doubles are written with 17 significant digits, so a write -> read round trip gives
// the identical model bit for bit.
#include "gripper_mi355x.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <string>
#include <vector>

void gm_derive_model_constants(gm_model* m);
void gm_derive_invweights(gm_model* m);

namespace {

// ------------------------------------------------------------------ minimal XML
struct XNode {
  std::string tag;
  std::vector<std::pair<std::string, std::string>> attr;
  std::vector<std::unique_ptr<XNode>> kids;
  const std::string* get(const char* k) const {
    for (auto& a : attr) if (a.first == k) return &a.second;
    return nullptr;
  }
};

struct XParser {
  const char* s;
  size_t i = 0, n;
  std::string err;
  explicit XParser(const char* src) : s(src), n(std::strlen(src)) {}
  void ws() { while (i < n && (s[i] == ' ' || s[i] == '\t' || s[i] == '\n' || s[i] == '\r')) i++; }
  bool skip_misc() {   // comments, declarations, processing instructions, text
    for (;;) {
      while (i < n && s[i] != '<') i++;
      if (i >= n) return false;
      if (std::strncmp(s + i, "<!--", 4) == 0) {
        const char* e = std::strstr(s + i + 4, "-->");
        if (!e) { err = "unterminated comment"; return false; }
        i = (size_t)(e - s) + 3;
      } else if (s[i + 1] == '?' || s[i + 1] == '!') {
        while (i < n && s[i] != '>') i++;
        i++;
      } else {
        return true;
      }
    }
  }
  std::unique_ptr<XNode> element() {
    if (!skip_misc()) return nullptr;
    if (s[i + 1] == '/') return nullptr;            // a closing tag: caller handles it
    i++;
    auto node = std::make_unique<XNode>();
    while (i < n && !std::strchr(" \t\r\n/>", s[i])) node->tag += s[i++];
    for (;;) {
      ws();
      if (i >= n) { err = "unterminated tag <" + node->tag; return nullptr; }
      if (s[i] == '/') {
        if (i + 1 < n && s[i + 1] == '>') { i += 2; return node; }
        err = "bad tag <" + node->tag; return nullptr;
      }
      if (s[i] == '>') { i++; break; }
      std::string k, v;
      while (i < n && !std::strchr(" \t\r\n=/>", s[i])) k += s[i++];
      ws();
      if (i >= n || s[i] != '=') { err = "attribute without value in <" + node->tag; return nullptr; }
      i++;
      ws();
      const char q = s[i];
      if (q != '"' && q != '\'') { err = "unquoted attribute in <" + node->tag; return nullptr; }
      i++;
      while (i < n && s[i] != q) v += s[i++];
      i++;
      node->attr.emplace_back(k, v);
    }
    for (;;) {
      auto kid = element();
      if (kid) { node->kids.push_back(std::move(kid)); continue; }
      if (!err.empty()) return nullptr;
      if (i >= n) { err = "missing </" + node->tag + ">"; return nullptr; }
      // closing tag
      size_t j = i + 2;
      std::string ct;
      while (j < n && s[j] != '>') ct += s[j++];
      while (!ct.empty() && std::strchr(" \t\r\n", ct.back())) ct.pop_back();
      if (ct != node->tag) { err = "mismatched </" + ct + "> for <" + node->tag + ">"; return nullptr; }
      i = j + 1;
      return node;
    }
  }
};

std::vector<double> nums(const std::string* v) {
  std::vector<double> out;
  if (!v) return out;
  const char* p = v->c_str();
  char* e;
  for (;;) {
    while (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r') p++;
    if (!*p) break;
    double x = std::strtod(p, &e);
    if (e == p) break;
    out.push_back(x);
    p = e;
  }
  return out;
}

// ------------------------------------------------------------------ writer
struct W {
  std::string out;
  int depth = 0;
  void line(const std::string& l) { out.append(2 * depth, ' '); out += l; out += '\n'; }
};
std::string f17(double x) { char b[40]; std::snprintf(b, sizeof b, "%.17g", x); return b; }
std::string vec(const double* v, int n) {
  std::string s;
  for (int k = 0; k < n; k++) { if (k) s += ' '; s += f17(v[k]); }
  return s;
}

const char* geom_type_name(int t) {
  switch (t) {
    case GM_GEOM_PLANE: return "plane";
    case GM_GEOM_SPHERE: return "sphere";
    case GM_GEOM_CAPSULE: return "capsule";
    case GM_GEOM_CYLINDER: return "cylinder";
    default: return "box";
  }
}
int geom_type_of(const std::string& s) {
  if (s == "plane") return GM_GEOM_PLANE;
  if (s == "sphere") return GM_GEOM_SPHERE;
  if (s == "capsule") return GM_GEOM_CAPSULE;
  if (s == "cylinder") return GM_GEOM_CYLINDER;
  if (s == "box") return GM_GEOM_BOX;
  return -1;
}

// reference names (JointSettings::Names, myfunctions.cpp:176-196; objecthandler.cpp)
struct Names {
  const gm_model* m;
  std::vector<std::string> body, joint, geom;
  explicit Names(const gm_model* mm) : m(mm) {
    body.assign(m->nbody, ""); joint.assign(m->njnt, ""); geom.assign(m->ngeom, "");
    body[0] = "world";
    body[m->body_base] = "gripper_base_link";
    body[m->body_palm] = "palm";
    body[m->body_obj] = "object";
    for (int f = 0; f < 3; f++) {
      const std::string F = "finger_" + std::to_string(f + 1);
      const int bint = m->dof_body[m->dof_pris[f]];
      body[bint] = F + "_intermediate";
      body[m->body_finger[f]] = F;
      for (int k = 1; k <= m->n_seg; k++) body[m->body_finger[f] + k] = F + "_segment_link_" + std::to_string(k + 1);
      joint[m->body_jnt[bint]] = F + "_prismatic_joint";
      joint[m->body_jnt[m->body_finger[f]]] = F + "_revolute_joint";
      for (int k = 1; k <= m->n_seg; k++) joint[m->body_jnt[m->body_finger[f] + k]] = F + "_segment_joint_" + std::to_string(k);
    }
    joint[m->body_jnt[m->body_base]] = "world_to_base";
    joint[m->body_jnt[m->body_palm]] = "palm_prismatic_joint";
    joint[m->body_jnt[m->body_obj]] = "object_freejoint";
    int cnt[8] = {0};
    for (int g = 0; g < m->ngeom; g++) {
      const int c = m->geom_class[g];
      std::string base;
      switch (c) {
        case GM_CLS_FINGER1: case GM_CLS_FINGER2: case GM_CLS_FINGER3:
          base = "finger_" + std::to_string(c) + "_geom_"; break;
        case GM_CLS_PALM: base = "palm_geom_"; break;
        case GM_CLS_GROUND: base = "ground_geom_"; break;
        case GM_CLS_OBJECT: base = "object_geom_"; break;
        default: base = "geom_"; break;
      }
      geom[g] = base + std::to_string(cnt[c & 7]++);
    }
  }
};

void write_body(W& w, const gm_model* m, const Names& nm, int b) {
  w.line("<body name=\"" + nm.body[b] + "\" pos=\"" + vec(m->body_pos[b], 3) + "\" quat=\"" + vec(m->body_quat[b], 4) + "\">");
  w.depth++;
  const int j = m->body_jnt[b];
  if (j >= 0) {
    if (m->jnt_type[j] == GM_JNT_FREE) {
      w.line("<freejoint name=\"" + nm.joint[j] + "\"/>");
    } else {
      const char* type = m->jnt_type[j] == GM_JNT_SLIDE ? "slide" : "hinge";
      w.line(std::string("<joint name=\"") + nm.joint[j] + "\" type=\"" + type + "\" pos=\"" + vec(m->jnt_pos[j], 3) +
             "\" axis=\"" + vec(m->jnt_axis[j], 3) + "\" stiffness=\"" + f17(m->jnt_stiffness[j]) + "\" damping=\"" +
             f17(m->jnt_damping[j]) + "\" armature=\"" + f17(m->jnt_armature[j]) + "\"/>");
    }
  }
  w.line("<inertial pos=\"" + vec(m->body_ipos[b], 3) + "\" mass=\"" + f17(m->body_mass[b]) + "\" diaginertia=\"" +
         vec(m->body_inertia[b], 3) + "\"/>");
  for (int g = 0; g < m->ngeom; g++) {
    if (m->geom_body[g] != b) continue;
    w.line("<geom name=\"" + nm.geom[g] + "\" type=\"" + geom_type_name(m->geom_type[g]) + "\" size=\"" +
           vec(m->geom_size[g], 3) + "\" pos=\"" + vec(m->geom_pos[g], 3) + "\" quat=\"" + vec(m->geom_quat[g], 4) +
           "\" friction=\"" + f17(m->geom_friction[g]) + " 0.005 0.0001\"/>");
  }
  for (int c = 0; c < m->nbody; c++)
    if (m->body_parent[c] == b && c != b) write_body(w, m, nm, c);
  w.depth--;
  w.line("</body>");
}

}  // namespace

extern "C" {

int64_t gm_model_to_mjcf(const gm_model* m, char* buf, int64_t cap) {
  if (!m) return GM_E_ARG;
  Names nm(m);
  W w;
  w.line("<!-- gripper-mi355x: the compiled gripper model as MJCF (gm_model_to_mjcf) -->");
  w.line("<mujoco model=\"gripper_mi355x\">");
  w.depth++;
  w.line("<compiler angle=\"radian\"/>");
  w.line("<option timestep=\"" + f17(m->timestep) + "\" gravity=\"" + vec(m->gravity, 3) + "\" solver=\"PGS\" iterations=\"" +
         std::to_string(m->pgs_iterations) + "\" mpr_tolerance=\"" + f17(m->mpr_tolerance) + "\" mpr_iterations=\"" +
         std::to_string(m->mpr_iterations) + "\"/>");
  w.line("<default>");
  w.depth++;
  w.line("<geom solref=\"" + vec(m->solref, 2) + "\" solimp=\"" + vec(m->solimp, 5) + "\"/>");
  w.depth--;
  w.line("</default>");
  // read_gripper_dimensions numerics (myfunctions.cpp:836-953), plus the per-finger tip
  // load direction used by the gauge calibration (apply_segment_force)
  w.line("<custom>");
  w.depth++;
  auto numeric = [&](const char* n, double v) { w.line(std::string("<numeric name=\"") + n + "\" data=\"" + f17(v) + "\"/>"); };
  numeric("finger_length", m->finger_length);
  numeric("finger_width", m->finger_width);
  numeric("finger_thickness", m->finger_thickness);
  numeric("finger_E", m->finger_E);
  numeric("fingertip_clearance", m->fingertip_clearance);
  numeric("hook_angle_degrees", m->hook_angle_degrees);
  numeric("hook_length", m->hook_length);
  numeric("fixed_hook_segment", 1);
  numeric("fixed_first_segment", m->fixed_first_segment);
  numeric("xy_base_joint", 0);
  numeric("xy_base_rotation", 0);
  numeric("z_base_rotation", 0);
  for (int f = 0; f < 3; f++)
    w.line("<numeric name=\"finger_" + std::to_string(f + 1) + "_tip_load_direction\" size=\"3\" data=\"" +
           vec(m->tip_dir[f], 3) + "\"/>");
  w.depth--;
  w.line("</custom>");
  w.line("<worldbody>");
  w.depth++;
  for (int g = 0; g < m->ngeom; g++) {
    if (m->geom_body[g] != 0) continue;
    w.line("<geom name=\"" + nm.geom[g] + "\" type=\"" + geom_type_name(m->geom_type[g]) + "\" size=\"" +
           vec(m->geom_size[g], 3) + "\" pos=\"" + vec(m->geom_pos[g], 3) + "\" quat=\"" + vec(m->geom_quat[g], 4) +
           "\" friction=\"" + f17(m->geom_friction[g]) + " 0.005 0.0001\"/>");
  }
  for (int b = 1; b < m->nbody; b++)
    if (m->body_parent[b] == 0) write_body(w, m, nm, b);
  w.depth--;
  w.line("</worldbody>");
  // the reference's motors (luke::control writes ctrl[n + i], myfunctions.cpp:1912-2057):
  // MJCF <motor> actuators on the 8 actuated joints select MuJoCo's explicit actuator path
  if (m->mujoco_actuators) {
    w.line("<actuator>");
    w.depth++;
    for (int f = 0; f < 3; f++) {
      const int jp = m->body_jnt[m->dof_body[m->dof_pris[f]]], jr = m->body_jnt[m->dof_body[m->dof_rev[f]]];
      w.line("<motor name=\"" + nm.joint[jp] + "_motor\" joint=\"" + nm.joint[jp] + "\" gear=\"1\"/>");
      w.line("<motor name=\"" + nm.joint[jr] + "_motor\" joint=\"" + nm.joint[jr] + "\" gear=\"1\"/>");
    }
    for (int d : {m->dof_palm, m->dof_base}) {
      const int j = m->body_jnt[m->dof_body[d]];
      w.line("<motor name=\"" + nm.joint[j] + "_motor\" joint=\"" + nm.joint[j] + "\" gear=\"1\"/>");
    }
    w.depth--;
    w.line("</actuator>");
  }
  w.line("<contact>");
  w.depth++;
  for (int p = 0; p < m->npair; p++)
    w.line("<pair geom1=\"" + nm.geom[m->pair_a[p]] + "\" geom2=\"" + nm.geom[m->pair_b[p]] + "\"/>");
  w.depth--;
  w.line("</contact>");
  // the reference's weld motor locks (set_constraint, myfunctions.cpp:1177-1279) on the
  // 1-dof motors: joint equalities
  w.line("<equality>");
  w.depth++;
  for (int k = 0; k < m->nlock; k++) {
    const int j = m->body_jnt[m->dof_body[m->lock_dof[k]]];
    w.line("<joint name=\"" + nm.joint[j] + "_lock\" joint1=\"" + nm.joint[j] + "\"/>");
  }
  w.depth--;
  w.line("</equality>");
  w.line("<keyframe>");
  w.depth++;
  w.line("<key name=\"initial pose\" qpos=\"" + vec(m->qpos0, m->nq) + "\"/>");
  w.depth--;
  w.line("</keyframe>");
  w.depth--;
  w.line("</mujoco>");
  const int64_t len = (int64_t)w.out.size();
  if (buf && cap > len) std::memcpy(buf, w.out.c_str(), (size_t)len + 1);
  return len;
}

int gm_model_from_mjcf(const char* xml, gm_model* out, char* err, int err_cap) {
  auto fail = [&](const std::string& msg) {
    if (err && err_cap > 0) std::snprintf(err, (size_t)err_cap, "%s", msg.c_str());
    return GM_E_ARG;
  };
  if (!xml || !out) return fail("null argument");
  XParser P(xml);
  auto root = P.element();
  if (!root) return fail("XML: " + (P.err.empty() ? std::string("no root element") : P.err));
  if (root->tag != "mujoco") return fail("root element is <" + root->tag + ">, not <mujoco>");
  gm_model* m = out;
  std::memset(m, 0, sizeof(*m));
  std::map<std::string, int> body_id, joint_id, geom_id;
  std::map<std::string, std::vector<double>> numeric;
  const XNode* world = nullptr;
  const XNode* contact = nullptr;
  const XNode* equality = nullptr;
  const XNode* keyframe = nullptr;
  m->timestep = 0.002; m->gravity[2] = -9.81;
  m->solref[0] = 0.02; m->solref[1] = 1.0;
  const double solimp_d[5] = {0.9, 0.95, 0.001, 0.5, 2.0};
  for (int k = 0; k < 5; k++) m->solimp[k] = solimp_d[k];
  m->pgs_iterations = 100; m->mpr_tolerance = 1e-6; m->mpr_iterations = 50;
  for (auto& kid : root->kids) {
    const XNode& x = *kid;
    if (x.tag == "option") {
      if (auto v = x.get("timestep")) m->timestep = std::strtod(v->c_str(), nullptr);
      auto g = nums(x.get("gravity"));
      if (g.size() == 3) for (int k = 0; k < 3; k++) m->gravity[k] = g[k];
      if (auto v = x.get("iterations")) m->pgs_iterations = std::atoi(v->c_str());
      if (auto v = x.get("mpr_tolerance")) m->mpr_tolerance = std::strtod(v->c_str(), nullptr);
      if (auto v = x.get("mpr_iterations")) m->mpr_iterations = std::atoi(v->c_str());
    } else if (x.tag == "default") {
      for (auto& d : x.kids) {
        if (d->tag != "geom") continue;
        auto sr = nums(d->get("solref")), si = nums(d->get("solimp"));
        if (sr.size() == 2) { m->solref[0] = sr[0]; m->solref[1] = sr[1]; }
        if (si.size() == 5) for (int k = 0; k < 5; k++) m->solimp[k] = si[k];
      }
    } else if (x.tag == "custom") {
      for (auto& d : x.kids)
        if (d->tag == "numeric" && d->get("name")) numeric[*d->get("name")] = nums(d->get("data"));
    } else if (x.tag == "worldbody") world = &x;
    else if (x.tag == "contact") contact = &x;
    else if (x.tag == "equality") equality = &x;
    else if (x.tag == "keyframe") keyframe = &x;
    else if (x.tag == "actuator") {
      for (auto& a : x.kids) if (a->tag == "motor") m->mujoco_actuators = 1;
    }
  }
  if (!world) return fail("no <worldbody>");
  // body tree, depth-first in document order (MuJoCo's compiler order)
  std::string berr;
  std::vector<int> last_dof(GM_MAX_BODY, -1);
  auto add_geoms = [&](const XNode& bx, int b) -> bool {
    for (auto& g : bx.kids) {
      if (g->tag != "geom") continue;
      if (m->ngeom >= GM_MAX_GEOM) { berr = "too many geoms"; return false; }
      const int id = m->ngeom++;
      const std::string name = g->get("name") ? *g->get("name") : "";
      geom_id[name] = id;
      const int t = geom_type_of(g->get("type") ? *g->get("type") : "sphere");
      if (t < 0) { berr = "unsupported geom type in " + name; return false; }
      m->geom_type[id] = t;
      m->geom_body[id] = b;
      auto sz = nums(g->get("size")), ps = nums(g->get("pos")), qt = nums(g->get("quat")), fr = nums(g->get("friction"));
      for (int k = 0; k < 3; k++) m->geom_size[id][k] = k < (int)sz.size() ? sz[k] : 0.0;
      for (int k = 0; k < 3; k++) m->geom_pos[id][k] = k < (int)ps.size() ? ps[k] : 0.0;
      if (qt.size() == 4) for (int k = 0; k < 4; k++) m->geom_quat[id][k] = qt[k];
      else { m->geom_quat[id][0] = 1; }
      m->geom_friction[id] = fr.empty() ? 1.0 : fr[0];
      const double* s = m->geom_size[id];
      double rb = 0;
      if (t == GM_GEOM_BOX) rb = std::sqrt(s[0] * s[0] + s[1] * s[1] + s[2] * s[2]);
      else if (t == GM_GEOM_SPHERE) rb = s[0];
      else if (t == GM_GEOM_CYLINDER) rb = std::sqrt(s[0] * s[0] + s[1] * s[1]);
      else if (t == GM_GEOM_CAPSULE) rb = s[0] + s[1];
      m->geom_rbound[id] = rb;
      // Contact::check_involves name prefixes (objecthandler.h:117-129)
      int cls = GM_CLS_NONE;
      if (name.rfind("finger_1", 0) == 0) cls = GM_CLS_FINGER1;
      else if (name.rfind("finger_2", 0) == 0) cls = GM_CLS_FINGER2;
      else if (name.rfind("finger_3", 0) == 0) cls = GM_CLS_FINGER3;
      else if (name.rfind("palm", 0) == 0) cls = GM_CLS_PALM;
      else if (name.rfind("ground", 0) == 0) cls = GM_CLS_GROUND;
      else if (name.rfind("object", 0) == 0) cls = GM_CLS_OBJECT;
      m->geom_class[id] = cls;
    }
    return true;
  };
  int nfree = 0;   // free joints seen (nq / GM_MAX_QPOS checked as they are added)
  std::function<bool(const XNode&, int)> walk = [&](const XNode& bx, int parent) -> bool {
    if (m->nbody >= GM_MAX_BODY) { berr = "too many bodies"; return false; }
    const int b = m->nbody++;
    const std::string name = bx.get("name") ? *bx.get("name") : "";
    body_id[name] = b;
    m->body_parent[b] = parent;
    m->body_jnt[b] = -1;
    auto ps = nums(bx.get("pos")), qt = nums(bx.get("quat"));
    for (int k = 0; k < 3; k++) m->body_pos[b][k] = k < (int)ps.size() ? ps[k] : 0.0;
    if (qt.size() == 4) for (int k = 0; k < 4; k++) m->body_quat[b][k] = qt[k];
    else m->body_quat[b][0] = 1;
    // group: JointSettings names (finger_N..., palm, gripper_base_link) / the free object
    int grp = m->body_group[parent];
    if (name.rfind("finger_1", 0) == 0) grp = GM_GRP_FINGER0;
    else if (name.rfind("finger_2", 0) == 0) grp = GM_GRP_FINGER0 + 1;
    else if (name.rfind("finger_3", 0) == 0) grp = GM_GRP_FINGER0 + 2;
    else if (name == "palm") grp = GM_GRP_PALM;
    else if (name == "gripper_base_link") grp = GM_GRP_BASE;
    for (auto& k : bx.kids) if (k->tag == "freejoint") grp = GM_GRP_OBJECT;
    m->body_group[b] = grp;
    last_dof[b] = last_dof[parent];
    for (auto& k : bx.kids) {
      const XNode& x = *k;
      if (x.tag == "inertial") {
        auto ip = nums(x.get("pos")), di = nums(x.get("diaginertia"));
        for (int q = 0; q < 3; q++) m->body_ipos[b][q] = q < (int)ip.size() ? ip[q] : 0.0;
        for (int q = 0; q < 3; q++) m->body_inertia[b][q] = q < (int)di.size() ? di[q] : 0.0;
        m->body_mass[b] = x.get("mass") ? std::strtod(x.get("mass")->c_str(), nullptr) : 0.0;
      } else if (x.tag == "joint" || x.tag == "freejoint") {
        if (m->body_jnt[b] >= 0) { berr = "body " + name + " has more than one joint"; return false; }
        const int j = m->njnt++;
        const std::string jn = x.get("name") ? *x.get("name") : "";
        joint_id[jn] = j;
        int type = GM_JNT_FREE;
        if (x.tag == "joint") {
          const std::string t = x.get("type") ? *x.get("type") : "hinge";
          type = t == "slide" ? GM_JNT_SLIDE : t == "hinge" ? GM_JNT_HINGE : t == "free" ? GM_JNT_FREE : -1;
          if (type < 0) { berr = "unsupported joint type " + t; return false; }
        }
        m->body_jnt[b] = j;
        m->jnt_type[j] = type;
        m->jnt_body[j] = b;
        m->jnt_qposadr[j] = m->nq;
        m->jnt_dofadr[j] = m->nv;
        auto jp = nums(x.get("pos")), ax = nums(x.get("axis"));
        for (int q = 0; q < 3; q++) m->jnt_pos[j][q] = q < (int)jp.size() ? jp[q] : 0.0;
        if (ax.size() == 3) for (int q = 0; q < 3; q++) m->jnt_axis[j][q] = ax[q];
        else if (type != GM_JNT_FREE) m->jnt_axis[j][2] = 1;
        m->jnt_stiffness[j] = x.get("stiffness") ? std::strtod(x.get("stiffness")->c_str(), nullptr) : 0.0;
        m->jnt_damping[j] = x.get("damping") ? std::strtod(x.get("damping")->c_str(), nullptr) : 0.0;
        m->jnt_armature[j] = x.get("armature") ? std::strtod(x.get("armature")->c_str(), nullptr) : 0.0;
        const int ndof = type == GM_JNT_FREE ? 6 : 1;
        if (type == GM_JNT_FREE && ++nfree > 1) { berr = "more than one free joint (the kernels hold one live object)"; return false; }
        if (m->nq + (type == GM_JNT_FREE ? 7 : 1) > GM_MAX_QPOS) { berr = "too many qpos"; return false; }
        m->nq += type == GM_JNT_FREE ? 7 : 1;
        for (int q = 0; q < ndof; q++) {
          if (m->nv >= GM_MAX_DOF) { berr = "too many dofs"; return false; }
          const int d = m->nv++;
          m->dof_parent[d] = q == 0 ? last_dof[parent] : d - 1;
          m->dof_body[d] = b;
          m->dof_group[d] = grp;
        }
        last_dof[b] = m->nv - 1;
      }
    }
    if (!add_geoms(bx, b)) return false;
    for (auto& k : bx.kids)
      if (k->tag == "body" && !walk(*k, b)) return false;
    return true;
  };
  // world body 0 and its geoms, then the bodies
  m->nbody = 1;
  m->body_parent[0] = -1;
  m->body_jnt[0] = -1;
  m->body_group[0] = GM_GRP_WORLD;
  m->body_quat[0][0] = 1;
  body_id["world"] = 0;
  if (!add_geoms(*world, 0)) return fail(berr);
  for (auto& k : world->kids)
    if (k->tag == "body" && !walk(*k, 0)) return fail(berr);
  // named indices (JointSettings, myfunctions.cpp:176-196, 719-787)
  auto J = [&](const std::string& n) { auto it = joint_id.find(n); return it == joint_id.end() ? -1 : it->second; };
  auto B = [&](const std::string& n) { auto it = body_id.find(n); return it == body_id.end() ? -1 : it->second; };
  const int jb = J("world_to_base"), jp = J("palm_prismatic_joint"), jo = J("object_freejoint");
  if (jb < 0 || jp < 0 || jo < 0) return fail("missing world_to_base / palm_prismatic_joint / object_freejoint");
  m->dof_base = m->jnt_dofadr[jb];
  m->dof_palm = m->jnt_dofadr[jp];
  m->dof_obj = m->jnt_dofadr[jo];
  m->body_base = B("gripper_base_link");
  m->body_palm = B("palm");
  m->body_obj = m->jnt_body[jo];
  if (m->body_base < 0 || m->body_palm < 0) return fail("missing gripper_base_link / palm bodies");
  int nseg = 0;
  while (J("finger_1_segment_joint_" + std::to_string(nseg + 1)) >= 0) nseg++;
  if (nseg < 1 || nseg > GM_MAX_SEG) return fail("finger segment joints: found " + std::to_string(nseg));
  m->n_seg = nseg;
  for (int f = 0; f < 3; f++) {
    const std::string F = "finger_" + std::to_string(f + 1);
    const int jpr = J(F + "_prismatic_joint"), jr = J(F + "_revolute_joint"), js = J(F + "_segment_joint_1"),
              jl = J(F + "_segment_joint_" + std::to_string(nseg));
    if (jpr < 0 || jr < 0 || js < 0 || jl < 0) return fail("missing joints of " + F);
    m->dof_pris[f] = m->jnt_dofadr[jpr];
    m->dof_rev[f] = m->jnt_dofadr[jr];
    m->dof_seg[f] = m->jnt_dofadr[js];
    m->body_finger[f] = B(F);
    if (m->body_finger[f] < 0) return fail("missing body " + F);
    m->body_tip[f] = m->jnt_body[jl];
    auto td = numeric.find(F + "_tip_load_direction");
    if (td != numeric.end() && td->second.size() == 3) for (int k = 0; k < 3; k++) m->tip_dir[f][k] = td->second[k];
  }
  // geoms: the live object's and the ground's
  m->geom_obj = m->geom_ground = -1;
  for (int g = 0; g < m->ngeom; g++) {
    if (m->geom_body[g] == m->body_obj && m->geom_obj < 0) m->geom_obj = g;
    if (m->geom_class[g] == GM_CLS_GROUND && m->geom_ground < 0) m->geom_ground = g;
  }
  if (m->geom_obj < 0 || m->geom_ground < 0) return fail("missing object / ground geom");
  // compact dof slots (as gm_build_model)
  for (int d = 0; d < m->nv; d++) {
    const int g = m->dof_group[d];
    if (g == GM_GRP_OBJECT) m->dof_slot[d] = d - m->dof_obj;
    else if (g == GM_GRP_BASE || g == GM_GRP_PALM) m->dof_slot[d] = 0;
    else if (g >= 0 && g < 3) m->dof_slot[d] = d - m->dof_pris[g];
  }
  // contact pairs
  if (contact)
    for (auto& k : contact->kids) {
      if (k->tag != "pair") continue;
      auto a = k->get("geom1"), b2 = k->get("geom2");
      if (!a || !b2 || !geom_id.count(*a) || !geom_id.count(*b2)) return fail("contact pair with an unknown geom");
      if (m->npair >= GM_MAX_PAIR) return fail("too many contact pairs");
      m->pair_a[m->npair] = geom_id[*a];
      m->pair_b[m->npair] = geom_id[*b2];
      m->npair++;
    }
  // motor locks
  if (equality)
    for (auto& k : equality->kids) {
      if (k->tag != "joint" || !k->get("joint1")) continue;
      const int j = J(*k->get("joint1"));
      if (j < 0) return fail("equality on an unknown joint");
      if (m->nlock >= GM_MAX_LOCK) return fail("too many motor locks");
      const int d = m->jnt_dofadr[j];
      m->lock_dof[m->nlock] = d;
      m->lock_kind[m->nlock] = (d == m->dof_palm) ? 2 : (d == m->dof_rev[0] || d == m->dof_rev[1] || d == m->dof_rev[2]) ? 1 : 0;
      m->nlock++;
    }
  // keyframe "initial pose" (myfunctions.cpp:171)
  if (keyframe)
    for (auto& k : keyframe->kids) {
      if (k->tag != "key" || !k->get("name") || *k->get("name") != "initial pose") continue;
      auto q = nums(k->get("qpos"));
      if ((int)q.size() != m->nq) return fail("keyframe qpos has the wrong size");
      for (int i = 0; i < m->nq; i++) m->qpos0[i] = q[i];
    }
  // gripper numerics (read_gripper_dimensions) and what the reference derives from them
  auto num = [&](const char* n, double dflt) {
    auto it = numeric.find(n);
    return (it != numeric.end() && !it->second.empty()) ? it->second[0] : dflt;
  };
  m->finger_length = num("finger_length", 235e-3);
  m->finger_width = num("finger_width", 28e-3);
  m->finger_thickness = num("finger_thickness", 0.9e-3);
  m->finger_E = num("finger_E", 193e9);
  m->fingertip_clearance = num("fingertip_clearance", 10e-3);
  m->hook_angle_degrees = num("hook_angle_degrees", 90.0);
  m->hook_length = num("hook_length", 35e-3);
  m->fixed_first_segment = (int32_t)num("fixed_first_segment", 0);
  if (m->nq > GM_MAX_QPOS) return fail("too many qpos");
  gm_derive_model_constants(m);
  gm_derive_invweights(m);
  return GM_OK;
}

}  // extern "C"
