// compat/rtnw_compat.h — brings the host API into the global namespace under the
// reference's names, so existing scene-builder code (main.cpp:49-230) compiles
// unchanged.  drand48 is deliberately NOT re-exported: builders keep calling libc
// drand48(), which is the stream rtnw::reset_reference_rng() positions.
#pragma once
#include <cfloat>
#include <cmath>
#include <cstdlib>
#include "../rtnw.h"

#ifndef MAXFLOAT
#define MAXFLOAT 0x1.fffffep+127f
#endif

using rtnw::vec3;
using rtnw::ray;
using rtnw::aabb;
using rtnw::ffmin;
using rtnw::ffmax;
using rtnw::surrounding_box;
using rtnw::dot;
using rtnw::cross;
using rtnw::unit_vector;
using rtnw::camera;
using rtnw::texture;
using rtnw::constant_texture;
using rtnw::checker_texture;
using rtnw::noise_texture;
using rtnw::image_texture;
using rtnw::perlin;
using rtnw::material;
using rtnw::lambertian;
using rtnw::metal;
using rtnw::dielectric;
using rtnw::diffuse_light;
using rtnw::isotropic;
using rtnw::hitable;
using rtnw::hitable_list;
using rtnw::sphere;
using rtnw::moving_sphere;
using rtnw::xy_rect;
using rtnw::xz_rect;
using rtnw::yz_rect;
using rtnw::box;
using rtnw::flip_normals;
using rtnw::translate;
using rtnw::rotate_y;
using rtnw::constant_medium;
using rtnw::bvh_node;
using rtnw::stbi_load;
