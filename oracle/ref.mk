# oracle/ref.mk — TEST INFRASTRUCTURE: builds the reference's own hot-path sources, where they lie
# under /root/reference (read-only), into oracle/_ref/ref_driver. Nothing is copied into the repo.
# Flags are the reference's own (CGL/CMakeLists.txt:46-61,148; CGL/find_avx.cmake:79-89):
#   -std=c++11 -m64 -fPIC -O3 -mavx2. -DGLEW_NO_GLU only tells the vendored glew.h not to include
# <GL/glu.h>; the one reference TU that calls GLU (src/application/application.cpp) is not built —
# ref_driver.cpp restates its scene-assembly glue instead.
# Usage: make -f oracle/ref.mk -j8        (outputs only under oracle/_ref/)

R    ?= /root/reference
OUT  ?= oracle/_ref
CXX  ?= g++
CC   ?= gcc
INC  := -I$(R)/CGL/include/CGL -I$(R)/src -I$(R)/CGL/include -I$(R)/CGL/deps/glew/include \
        -I$(R)/CGL/deps/glfw/include -I$(R)/src/imgui -I$(R)/src/imgui/backends
CXXFLAGS := -std=c++11 -m64 -fPIC -O3 -mavx2 -DGLEW_NO_GLU -w $(INC)

SRCS := src/pathtracer/bidirection.cpp src/pathtracer/pathtracer.cpp src/pathtracer/bsdf.cpp \
        src/pathtracer/advanced_bsdf.cpp src/pathtracer/sampler.cpp src/pathtracer/camera.cpp \
        src/pathtracer/camera_lens.cpp src/pathtracer/raytraced_renderer.cpp \
        src/scene/bvh.cpp src/scene/bbox.cpp src/scene/triangle.cpp src/scene/sphere.cpp \
        src/scene/light.cpp src/scene/environment_light.cpp src/scene/object.cpp \
        $(wildcard $(R)/src/scene/collada/*.cpp) \
        src/scene/gl_scene/mesh.cpp src/scene/gl_scene/scene.cpp src/scene/gl_scene/sphere.cpp \
        src/util/halfEdgeMesh.cpp src/util/sphere_drawing.cpp src/application/visual_debugger.cpp \
        src/application/meshEdit.cpp \
        CGL/src/vector2D.cpp CGL/src/vector3D.cpp CGL/src/vector4D.cpp CGL/src/matrix3x3.cpp \
        CGL/src/matrix4x4.cpp CGL/src/tinyxml2.cpp CGL/src/lodepng.cpp CGL/src/color.cpp \
        CGL/src/complex.cpp CGL/src/quaternion.cpp CGL/src/base64.cpp CGL/src/path.cpp \
        src/imgui/imgui.cpp src/imgui/imgui_widgets.cpp src/imgui/imgui_draw.cpp src/imgui/imgui_tables.cpp
SRCS := $(patsubst $(R)/%,%,$(SRCS))
OBJS := $(addprefix $(OUT)/obj/,$(SRCS:.cpp=.o))

all: $(OUT)/ref_driver $(OUT)/ref_env_kat

$(OUT)/obj/%.o: $(R)/%.cpp
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -c $< -o $@

$(OUT)/obj/glew.o: $(R)/CGL/deps/glew/src/glew.c
	@mkdir -p $(dir $@)
	$(CC) -O2 -fPIC -DGLEW_NO_GLU -I$(R)/CGL/deps/glew/include -w -c $< -o $@

$(OUT)/obj/ref_driver.o: oracle/ref_driver.cpp
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -c $< -o $@

$(OUT)/ref_driver: $(OBJS) $(OUT)/obj/glew.o $(OUT)/obj/ref_driver.o
	$(CXX) -o $@ $^ -lGL -lpthread

# integration check (tests/test_integration.py): ref_driver with the reference-side binding
# integration/bidirection_amd.h swapped in for BidirectionalPathTracer (-G), linked to the product
# library. `make -f oracle/ref.mk amd` after libbdpt_amd.so is built.
LIBDIR := bidirectional-pathtracing_amd
$(OUT)/obj/ref_driver_amd.o: oracle/ref_driver.cpp integration/bidirection_amd.h include/bdpt/bdpt.h
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -DBDPT_INTEGRATION -Iinclude -Iintegration -c $< -o $@

$(OUT)/ref_driver_amd: $(OBJS) $(OUT)/obj/glew.o $(OUT)/obj/ref_driver_amd.o $(LIBDIR)/libbdpt_amd.so
	$(CXX) -o $@ $(OBJS) $(OUT)/obj/glew.o $(OUT)/obj/ref_driver_amd.o -L$(LIBDIR) -l:libbdpt_amd.so \
	  -L/opt/rocm/lib -Wl,-rpath-link,/opt/rocm/lib -Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)' -lGL -lpthread

amd: $(OUT)/ref_driver_amd
.PHONY: all amd

# environment-light known answers (tests/test_env.py): EnvironmentLight + sampler + tinyexr
ENV_OBJS := $(addprefix $(OUT)/obj/,src/scene/environment_light.o src/pathtracer/sampler.o CGL/src/lodepng.o \
            CGL/src/vector2D.o CGL/src/vector3D.o CGL/src/vector4D.o CGL/src/matrix3x3.o CGL/src/matrix4x4.o \
            CGL/src/color.o CGL/src/complex.o CGL/src/quaternion.o)

$(OUT)/obj/ref_env_kat.o: oracle/ref_env_kat.cpp
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -c $< -o $@

$(OUT)/ref_env_kat: $(ENV_OBJS) $(OUT)/obj/ref_env_kat.o
	$(CXX) -o $@ $^ -lpthread

clean:
	rm -rf $(OUT)/obj $(OUT)/ref_driver $(OUT)/ref_env_kat

.PHONY: all clean
