package io.scalecube.cluster.sim;

import static io.scalecube.cluster.sim.SwimNative.call;
import static java.lang.foreign.ValueLayout.ADDRESS;
import static java.lang.foreign.ValueLayout.JAVA_INT;
import static java.lang.foreign.ValueLayout.JAVA_LONG;

import io.scalecube.cluster.ClusterConfig;
import io.scalecube.cluster.Member;
import io.scalecube.cluster.fdetector.FailureDetector;
import io.scalecube.cluster.fdetector.FailureDetectorEvent;
import io.scalecube.cluster.fdetector.SimFailureDetector;
import io.scalecube.cluster.gossip.GossipProtocol;
import io.scalecube.cluster.gossip.SimGossipProtocol;
import io.scalecube.cluster.membership.MemberStatus;
import io.scalecube.cluster.membership.MembershipEvent;
import io.scalecube.cluster.membership.MembershipProtocol;
import io.scalecube.cluster.membership.SimMembershipProtocol;
import io.scalecube.cluster.transport.api.Message;
import io.scalecube.net.Address;
import java.lang.foreign.Arena;
import java.lang.foreign.MemorySegment;
import java.nio.ByteBuffer;
import java.time.Duration;
import java.util.ArrayList;
import java.util.HashMap;
import java.util.List;
import java.util.Map;
import java.util.Optional;
import java.util.TreeSet;
import java.util.concurrent.Callable;
import reactor.core.publisher.DirectProcessor;
import reactor.core.publisher.FluxSink;
import reactor.core.publisher.Mono;
import reactor.core.publisher.MonoProcessor;
import reactor.core.scheduler.Scheduler;
import reactor.core.scheduler.Schedulers;

/**
 * A whole simulated cluster on one MI355X: replaces N x {@code ClusterImpl.doStart0}'s protocol
 * wiring (ClusterImpl.java:260-291 constructs FailureDetectorImpl, GossipProtocolImpl,
 * MetadataStoreImpl and MembershipProtocolImpl per member) with one libswimgpu engine, and hands out
 * per-member views implementing the reference's own protocol interfaces. Virtual time advances only
 * in {@link #advance}; events the engine emitted are then republished into each member's
 * DirectProcessor in the engine's canonical order (tick, viewer, phase, minor), on the cluster's
 * single scheduler thread (the engine handle is single-threaded, like the reference's per-member
 * {@code publishOn(scheduler)} confinement, ClusterImpl.java:257).
 *
 * <p>Members are slots 0..capacity-1; member s has id "sim-s" and, unless it was started on the
 * address of a stopped member ({@link #startOnAddressOf}), address sim:(basePort + s).
 */
public final class SimulatedCluster implements AutoCloseable {
  private static final int EVENT_BATCH = 1 << 16;
  private static final int BASE_PORT = 20000;

  private final Arena arena = Arena.ofShared();
  private final MemorySegment engine;
  private final int capacity;
  private final int tickMs;
  private final String namespace;
  private final Scheduler scheduler = Schedulers.newSingle("swimgpu-sim", true);
  private final MemorySegment events;
  private final MemorySegment row;
  private final int[] addressSlot;
  private final long[] metadataVersion;
  // per member: the destinations / sources it holds NetworkEmulator link overrides for, so that
  // blockAll* / unblockAll* can clear them (outboundSettings.clear(), NetworkEmulator.java:88-99,238-249)
  private final Map<Integer, TreeSet<Integer>> outLinks = new HashMap<>();
  private final Map<Integer, TreeSet<Integer>> inLinks = new HashMap<>();

  private final List<DirectProcessor<MembershipEvent>> membership = new ArrayList<>();
  private final List<FluxSink<MembershipEvent>> membershipSinks = new ArrayList<>();
  private final List<DirectProcessor<FailureDetectorEvent>> fd = new ArrayList<>();
  private final List<FluxSink<FailureDetectorEvent>> fdSinks = new ArrayList<>();
  private final List<DirectProcessor<Message>> gossips = new ArrayList<>();
  private final List<FluxSink<Message>> gossipSinks = new ArrayList<>();

  // user gossip payloads travel the engine as 32-bit handles (swim_spread); spread() futures wait
  // for SWIM_EV_SPREAD_DONE of (originator, handle)
  private final Map<Integer, Message> payloads = new HashMap<>();
  private final Map<Long, MonoProcessor<String>> spreadFutures = new HashMap<>();
  private int nextPayload = 1;

  private SimulatedCluster(MemorySegment engine, int capacity, int tickMs, String namespace) {
    this.engine = engine;
    this.capacity = capacity;
    this.tickMs = tickMs;
    this.namespace = namespace;
    this.events = arena.allocate(SwimNative.EVENT, EVENT_BATCH);
    this.row = arena.allocate(JAVA_LONG, capacity);
    this.addressSlot = new int[capacity];
    this.metadataVersion = new long[capacity];
    for (int s = 0; s < capacity; s++) {
      addressSlot[s] = s;
      DirectProcessor<MembershipEvent> m = DirectProcessor.create();
      membership.add(m);
      membershipSinks.add(m.sink());
      DirectProcessor<FailureDetectorEvent> f = DirectProcessor.create();
      fd.add(f);
      fdSinks.add(f.sink());
      DirectProcessor<Message> g = DirectProcessor.create();
      gossips.add(g);
      gossipSinks.add(g.sink());
    }
  }

  /**
   * A converged cluster of {@code initial} members (slots [0, initial)) in {@code capacity} slots;
   * the rest join later through the seeds. {@code seed} keys the engine's counter-based RNG.
   */
  public static SimulatedCluster create(ClusterConfig config, int capacity, int initial, long seed, int device) {
    Arena a = Arena.ofAuto();
    MemorySegment cfg = a.allocate(SwimNative.CONFIG);
    call(SwimNative.CONFIG_DEFAULT, "swim_config_default", cfg, 0);
    set(cfg, "ping_interval", config.failureDetectorConfig().pingInterval());
    set(cfg, "ping_timeout", config.failureDetectorConfig().pingTimeout());
    set(cfg, "ping_req_members", config.failureDetectorConfig().pingReqMembers());
    set(cfg, "gossip_interval", (int) config.gossipConfig().gossipInterval());
    set(cfg, "gossip_fanout", config.gossipConfig().gossipFanout());
    set(cfg, "gossip_repeat_mult", config.gossipConfig().gossipRepeatMult());
    set(cfg, "gossip_segmentation_threshold", config.gossipConfig().gossipSegmentationThreshold());
    set(cfg, "sync_interval", config.membershipConfig().syncInterval());
    set(cfg, "sync_timeout", config.membershipConfig().syncTimeout());
    set(cfg, "suspicion_mult", config.membershipConfig().suspicionMult());
    set(cfg, "removed_members_history_size", config.membershipConfig().removedMembersHistorySize());
    set(cfg, "metadata_timeout", config.metadataTimeout());
    set(cfg, "record_fd_events", 1);
    set(cfg, "device", device);
    MemorySegment out = a.allocate(ADDRESS);
    call(SwimNative.CREATE, "swim_create", cfg, capacity, initial, seed, out);
    MemorySegment e = out.get(ADDRESS, 0);
    MemorySegment now = a.allocate(JAVA_LONG);
    MemorySegment tick = a.allocate(JAVA_INT);
    MemorySegment tpp = a.allocate(JAVA_INT);
    call(SwimNative.NOW, "swim_now", e, now, tick, tpp);
    SimulatedCluster c = new SimulatedCluster(e, capacity, tick.get(JAVA_INT, 0), config.membershipConfig().namespace());
    List<Address> seeds = config.membershipConfig().seedMembers();
    if (!seeds.isEmpty()) {
      int[] slots = seeds.stream().mapToInt(ad -> ad.port() - BASE_PORT).toArray();
      MemorySegment sv = a.allocate(JAVA_INT, slots.length);
      for (int i = 0; i < slots.length; i++) sv.setAtIndex(JAVA_INT, i, slots[i]);
      call(SwimNative.SET_SEEDS, "swim_set_seeds", e, sv, slots.length);
    }
    return c;
  }

  private static void set(MemorySegment cfg, String field, int v) {
    cfg.set(JAVA_INT, SwimNative.CONFIG.byteOffset(java.lang.foreign.MemoryLayout.PathElement.groupElement(field)), v);
  }

  // ------------------------------------------------------------------ members and views
  public int capacity() { return capacity; }

  public Member member(int s) {
    return new Member("sim-" + s, null, Address.create("sim", BASE_PORT + addressSlot[s]), namespace);
  }

  public int slotOf(String id) { return Integer.parseInt(id.substring(4)); }

  public MembershipProtocol membership(int s) { return new SimMembershipProtocol(this, s); }

  public FailureDetector failureDetector(int s) { return new SimFailureDetector(this, s); }

  public GossipProtocol gossip(int s) { return new SimGossipProtocol(this, s); }

  public SimNetworkEmulator networkEmulator(int s) { return new SimNetworkEmulator(this, s); }

  public DirectProcessor<MembershipEvent> membershipEvents(int s) { return membership.get(s); }

  public DirectProcessor<FailureDetectorEvent> failureDetectorEvents(int s) { return fd.get(s); }

  public DirectProcessor<Message> gossipMessages(int s) { return gossips.get(s); }

  /** membershipTable of viewer s as swim.h cells (MembershipProtocolImpl.getMembershipRecords :903-905). */
  public long[] view(int s) {
    return onScheduler(() -> {
      call(SwimNative.READ_VIEW, "swim_read_view", engine, s, row);
      return row.toArray(JAVA_LONG);
    });
  }

  public Optional<MemberStatus> status(int viewer, int subject) {
    long c = view(viewer)[subject];
    return SwimNative.cellInTable(c) ? Optional.of(MemberStatus.values()[SwimNative.cellStatus(c)]) : Optional.empty();
  }

  // ------------------------------------------------------------------ lifecycle (ClusterImpl)
  /** ClusterImpl.start of a fresh member in free slot s: initial SYNC to every seed next tick. */
  public void start(int s) { run(() -> call(SwimNative.JOIN, "swim_join", engine, s)); }

  /**
   * ClusterImpl.start of a fresh member in free slot s with its own ClusterConfig: its
   * membershipConfig().seedMembers() become s's seed list (MembershipProtocolImpl :120-130,
   * cleanUpSeedMembers :171-190) — start0's initial SYNCs and selectSyncAddress use them.
   */
  public void start(int s, ClusterConfig config) {
    run(() -> {
      int[] slots = config.membershipConfig().seedMembers().stream().mapToInt(ad -> ad.port() - BASE_PORT).toArray();
      try (Arena a = Arena.ofConfined()) {
        MemorySegment sv = a.allocate(JAVA_INT, Math.max(1, slots.length));
        for (int i = 0; i < slots.length; i++) sv.setAtIndex(JAVA_INT, i, slots[i]);
        call(SwimNative.SET_MEMBER_SEEDS, "swim_set_member_seeds", engine, s, sv, slots.length);
      }
      call(SwimNative.JOIN, "swim_join", engine, s);
    });
  }

  /** A restart on the same port: s binds the address of stopped member `old` (DEST_GONE for `old`). */
  public void startOnAddressOf(int s, int old) {
    run(() -> call(SwimNative.JOIN_AT, "swim_join_at", engine, s, old));
    addressSlot[s] = addressSlot[old];
  }

  /** Transport stopped without leaving (the reference tests' stop / kill). */
  public void stop(int s) { run(() -> call(SwimNative.KILL, "swim_kill", engine, s)); }

  /** ClusterImpl.shutdown (:508-517): leaveCluster, stop once the LEAVING gossip has spread. */
  public void shutdown(int s) { run(() -> call(SwimNative.LEAVE, "swim_leave", engine, s, 1)); }

  /** ClusterImpl.updateMetadata (:497-500) -> updateIncarnation (:214-226); viewers see UPDATED. */
  public void updateMetadata(int s) {
    run(() -> call(SwimNative.UPDATE_METADATA, "swim_update_metadata", engine, s));
    metadataVersion[s]++;
  }

  // ------------------------------------------------------------------ virtual time
  /** Advance virtual time, then republish the events of that time span. */
  public Mono<Void> advance(Duration d) {
    int ticks = (int) Math.max(1, d.toMillis() / tickMs);
    return Mono.fromRunnable(() -> {
          call(SwimNative.STEP_TICKS, "swim_step_ticks", engine, ticks);
          pump();
        })
        .subscribeOn(scheduler)
        .then();
  }

  private void pump() {
    MemorySegment nOut = arena.allocate(JAVA_LONG);
    while (true) {
      call(SwimNative.DRAIN_EVENTS, "swim_drain_events", engine, events, (long) EVENT_BATCH, nOut);
      long n = nOut.get(JAVA_LONG, 0);
      for (long i = 0; i < n; i++) dispatch(events.asSlice(i * SwimNative.EVENT.byteSize(), SwimNative.EVENT));
      if (n < EVENT_BATCH) return;
    }
  }

  private void dispatch(MemorySegment ev) {
    final long tick = (long) SwimNative.EV_TICK.get(ev, 0L);
    final int viewer = (int) SwimNative.EV_VIEWER.get(ev, 0L);
    final int subject = (int) SwimNative.EV_SUBJECT.get(ev, 0L);
    final int type = (int) SwimNative.EV_TYPE.get(ev, 0L);
    final int data = (int) SwimNative.EV_DATA.get(ev, 0L);
    final long ts = tick * tickMs; // virtual ms (the reference stamps wall-clock ms)
    final Member m = member(subject);
    final ByteBuffer meta = ByteBuffer.allocate(Long.BYTES).putLong(0, metadataVersion[subject]);
    switch (type) {
      case SwimNative.EV_ADDED:
        membershipSinks.get(viewer).next(MembershipEvent.createAdded(m, meta, ts));
        break;
      case SwimNative.EV_REMOVED:
        membershipSinks.get(viewer).next(MembershipEvent.createRemoved(m, meta, ts));
        break;
      case SwimNative.EV_LEAVING:
        membershipSinks.get(viewer).next(MembershipEvent.createLeaving(m, meta, ts));
        break;
      case SwimNative.EV_UPDATED:
        membershipSinks.get(viewer).next(MembershipEvent.createUpdated(m, null, meta, ts));
        break;
      case SwimNative.EV_FD_ALIVE:
      case SwimNative.EV_FD_SUSPECT:
      case SwimNative.EV_FD_DEAD:
        fdSinks.get(viewer).next(SimFailureDetector.event(m, MemberStatus.values()[type == SwimNative.EV_FD_ALIVE
            ? 0 : type == SwimNative.EV_FD_SUSPECT ? 1 : 3]));
        break;
      case SwimNative.EV_GOSSIP: {
        Message msg = payloads.get(data);
        if (msg != null) gossipSinks.get(viewer).next(msg);
        break;
      }
      case SwimNative.EV_SPREAD_DONE: {
        MonoProcessor<String> done = spreadFutures.remove(key(viewer, data));
        if (done != null) done.onNext("sim-" + viewer + "-" + data);
        break;
      }
      default:
        break;
    }
  }

  // ------------------------------------------------------------------ user gossips
  /** GossipProtocol.spread (GossipProtocolImpl.java:126-130): the message stays here under a handle. */
  public Mono<String> spread(int s, Message message) {
    MonoProcessor<String> done = MonoProcessor.create();
    run(() -> {
      int h = nextPayload++;
      payloads.put(h, message);
      spreadFutures.put(key(s, h), done);
      call(SwimNative.SPREAD, "swim_spread", engine, s, h);
    });
    return done;
  }

  private static long key(int member, int handle) { return ((long) member << 32) | (handle & 0xffffffffL); }

  // ------------------------------------------------------------------ SYNC from outside the simulation
  /**
   * onSyncAck (MembershipProtocolImpl.java:363-391) at member {@code viewer} for a SyncData that arrived
   * from a real node (decoded by the caller's codec): its records in order, as (member slot, status,
   * incarnation) — swim_ingest_sync, {@code initial} for start0's INITIAL_SYNC reason.
   */
  public void ingestSync(int viewer, int[] members, int[] statuses, int[] incarnations, boolean initial) {
    if (members.length != statuses.length || members.length != incarnations.length) {
      throw new IllegalArgumentException("record arrays differ in length");
    }
    run(() -> {
      try (Arena a = Arena.ofConfined()) {
        MemorySegment recs = a.allocate(16L * Math.max(1, members.length), 16);  // swim_record: 4 x u32
        for (int i = 0; i < members.length; i++) {
          recs.setAtIndex(JAVA_INT, 4L * i, members[i]);
          recs.setAtIndex(JAVA_INT, 4L * i + 1, statuses[i]);
          recs.setAtIndex(JAVA_INT, 4L * i + 2, incarnations[i]);
          recs.setAtIndex(JAVA_INT, 4L * i + 3, 0);
        }
        call(SwimNative.INGEST_SYNC, "swim_ingest_sync", engine, viewer, recs, members.length, initial ? 1 : 0);
      }
    });
  }

  // ------------------------------------------------------------------ plumbing
  MemorySegment engine() { return engine; }

  /** OutboundSettings' loss is a percentage (NetworkEmulator.java:349-352); checked before any engine call */
  void checkLossPercent(int lossPercent) {
    if (lossPercent < 0 || lossPercent > 100) {
      throw new IllegalArgumentException("lossPercent must be within 0..100: " + lossPercent);
    }
  }

  void noteOutLink(int member, int destination) {
    outLinks.computeIfAbsent(member, k -> new TreeSet<>()).add(destination);
  }

  void noteInLink(int member, int source) {
    inLinks.computeIfAbsent(member, k -> new TreeSet<>()).add(source);
  }

  /** the member's link overrides, ascending; forgotten (the caller removes them from the engine) */
  int[] takeOutLinks(int member) {
    TreeSet<Integer> s = outLinks.remove(member);
    return s == null ? new int[0] : s.stream().mapToInt(Integer::intValue).toArray();
  }

  int[] takeInLinks(int member) {
    TreeSet<Integer> s = inLinks.remove(member);
    return s == null ? new int[0] : s.stream().mapToInt(Integer::intValue).toArray();
  }

  void run(Runnable r) {
    onScheduler(() -> {
      r.run();
      return null;
    });
  }

  <T> T onScheduler(Callable<T> c) {
    return Mono.fromCallable(c).subscribeOn(scheduler).block();
  }

  @Override
  public void close() {
    run(() -> call(SwimNative.DESTROY, "swim_destroy", engine));
    scheduler.dispose();
    arena.close();
  }
}
