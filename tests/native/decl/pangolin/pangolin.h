// Declaration-only stand-in (the reference's Map.h includes Pangolin but
// declares nothing against it) for the syntax check of
// adapters/orbslam3/ORBmatcher_searches.cc (tests/test_adapter.py).  Test
// infrastructure; it stands in for no part of the reference itself.
#pragma once
// the OpenGL types Pangolin's headers bring in (GL/gl.h)
typedef unsigned char GLubyte;
typedef unsigned int GLuint;
typedef int GLint;
typedef float GLfloat;
typedef double GLdouble;
namespace pangolin {
class OpenGlMatrix;
}
